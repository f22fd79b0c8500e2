#!/bin/bash
# Run ON THE GPU BOX: POA parity tests, the POA bench, and (if built) the phase-diagnostic
# variant svtrek_amd/variants/poa_diag.so.   tools/gpu_poa.sh TAG [extra bench_poa args]
set -u
TAG=${1:?tag}; shift
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/poa_$TAG
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_poa.py -x -v --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?
tail -3 "$OUT/tests.log"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python tools/bench_poa.py "$@" > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -5 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
if [ -f svtrek_amd/variants/poa_diag.so ]; then
  SVTREK_ENGINE_LIB=$PWD/svtrek_amd/variants/poa_diag.so timeout -k 10 400 python tools/bench_poa.py --repeat 1 \
    --cpu-sample 1 --check 3 "$@" > "$OUT/diag.json" 2> "$OUT/diag.err" || { tail -5 "$OUT/diag.err"; exit 1; }
  grep poa_diag "$OUT/diag.err" | tail -4
fi
