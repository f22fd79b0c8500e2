#!/bin/bash
# Build engine variants (compile-time knobs) into variants/NAME.so for an A/B bench on the
# GPU box (bench.py honours SVTREK_ENGINE_LIB).   tools/build_variants.sh NAME "-DKNOB=V ..." ...
set -eu
cd "$(dirname "$0")/.."
mkdir -p variants
while [ $# -ge 2 ]; do
  name=$1; defs=$2; shift 2
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -I include $defs \
    -o "variants/$name.so" svtrek_amd/csrc/svt_engine.hip -Rpass-analysis=kernel-resource-usage 2> "variants/$name.res" &
done
wait
for f in variants/*.res; do
  echo "== $f"; grep -A8 "index_kernel" "$f" | grep -E "Function Name|VGPRs:|Scratch" | sed 's/.*remark: *//; s/ \[-R.*//' | paste - - -
done
