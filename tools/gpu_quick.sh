#!/bin/bash
# Run ON THE GPU BOX: a parity subset (tests matching -k EXPR) + the default bench, one
# time limit per step, stopping at the first crash / timeout.   tools/gpu_quick.sh TAG [-k EXPR] [bench args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
TAG=${1:?tag}; shift
K="api or parity or workloads"
if [ "${1:-}" = "-k" ]; then K=$2; shift 2; fi
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
run() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] start $name" >> "$OUT/steps.log"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] end $name rc=$rc" >> "$OUT/steps.log"
  return $rc
}
run pytest 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K"; rc=$?
tail -3 "$OUT/pytest.log"
if [ $rc -gt 1 ]; then echo "pytest crashed rc=$rc"; exit $rc; fi
run bench 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline "$@" || exit $?
tail -1 "$OUT/bench.log"
export TMPDIR=/tmp
run trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
  python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-cold "$@" || exit $?
head -8 "$OUT/trace/run_kernel_stats.csv" | cut -c1-150
exit $rc
