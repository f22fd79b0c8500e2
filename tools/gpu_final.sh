#!/bin/bash
# Run ON THE GPU BOX: the round's closing measurements -- kernel trace + HBM PMC passes of
# bench.py (tools/gpu_profile.sh), the default bench line (with the CPU baseline), the POA
# bench and its kernel trace, and the end-to-end CLI timing.  Stops at the first failing step.
#   tools/gpu_final.sh TAG
set -u
TAG=${1:?tag}
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/final_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] $name" >> "$OUT/steps.log"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" >> "$OUT/steps.log"
  if [ $rc -ne 0 ]; then echo "step $name failed rc=$rc"; tail -20 "$OUT/$name.log"; exit $rc; fi
}
bash tools/gpu_profile.sh "$TAG" || exit $?
step bench 300 python3 bench.py
tail -1 "$OUT/bench.log"
step poa_bench 400 python3 tools/bench_poa.py
tail -1 "$OUT/poa_bench.log"
step poa_trace 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/poa_trace" -o run -- \
  python3 tools/bench_poa.py --repeat 1 --cpu-sample 1 --check 3
step e2e 400 python3 tools/e2e_bench.py
tail -1 "$OUT/e2e.log"
echo "final $TAG done"
