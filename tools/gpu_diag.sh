#!/bin/bash
# Run ON THE GPU BOX: bench only (no parity: diagnostic builds give wrong results) for the
# default engine and every library in svtrek_amd/variants/, each with the given bench args.
#   tools/gpu_diag.sh TAG "bench args 1" ["bench args 2" ...]
set -u
TAG=${1:?tag}; shift
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/diag_$TAG
mkdir -p "$OUT"
i=0
for lib in svtrek_amd/libsvtrek_hip.so svtrek_amd/diag/*.so; do
  name=$(basename "$lib" .so)
  for args in "$@"; do
    i=$((i+1))
    SVTREK_ENGINE_LIB=$PWD/$lib timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-verify $args > "$OUT/$i.log" 2>&1 || { echo "fail $name $args"; tail -5 "$OUT/$i.log"; exit 1; }
    echo "$name [$args] $(python3 -c "import json;d=json.loads(open('$OUT/$i.log').read().strip().splitlines()[-1]);r=d['roofline'];print(round(d['value']), r['kernel_ms_mean'], r['frac'])")" | tee -a "$OUT/summary.txt"
  done
done
