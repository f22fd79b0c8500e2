#!/bin/bash
# Run ON THE GPU BOX: parity subset + bench for every engine variant in svtrek_amd/variants/.
#   tools/gpu_variants.sh TAG [bench args...]
set -u
TAG=${1:?tag}; shift
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/var_$TAG
mkdir -p "$OUT"
for lib in svtrek_amd/libsvtrek_hip.so svtrek_amd/variants/*.so; do
  name=$(basename "$lib" .so)
  echo "[$(date +%T)] $name" >> "$OUT/steps.log"
  SVTREK_ENGINE_LIB=$PWD/$lib timeout -k 10 400 python -m pytest tests/test_gpu_parity.py -x -q > "$OUT/$name.pytest.log" 2>&1
  rc=$?; echo "  pytest rc=$rc" >> "$OUT/steps.log"
  if [ $rc -gt 1 ]; then echo "crash in $name"; exit $rc; fi
  SVTREK_ENGINE_LIB=$PWD/$lib timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline "$@" > "$OUT/$name.bench.log" 2>&1 || exit $?
  echo "$name $(tail -1 $OUT/$name.pytest.log) $(python3 -c "import json,sys;d=json.loads(open('$OUT/$name.bench.log').read().strip().splitlines()[-1]);r=d['roofline'];print(d['value'],r['kernel_ms_mean'],r['frac'])")"
done
