#!/bin/bash
# Run ON THE GPU BOX: smoke, every -m gpu test, the default bench line (with the CPU baseline),
# a kernel trace of the cfg4 step, then the cfg5 bench line and its trace.  One time limit per
# step; stops at the first crash / timeout.   tools/gpu_full.sh TAG [--no-cfg5]
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
TAG=${1:?tag}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] start $name" >> "$OUT/steps.log"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] end $name rc=$rc" >> "$OUT/steps.log"
  return $rc
}
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
run pytest 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread; rc=$?
tail -3 "$OUT/pytest.log"
if [ $rc -ne 0 ]; then echo "pytest rc=$rc"; exit $rc; fi
run bench 400 python bench.py --steps 20 --warmup 3 || exit $?
tail -1 "$OUT/bench.log" | cut -c1-300
run trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
  python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-cold || exit $?
head -8 "$OUT/trace/run_kernel_stats.csv" | cut -c1-150
[ "${1:-}" = "--no-cfg5" ] && exit 0
run cfg5 600 python -u bench.py --workload cfg5_100k_60x_ul_ont --steps 10 --warmup 2 --no-cpu-baseline || exit $?
tail -1 "$OUT/cfg5.log" | cut -c1-300
run trace5 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace5" -o run -- \
  python3 bench.py --workload cfg5_100k_60x_ul_ont --steps 5 --warmup 1 --no-cpu-baseline --no-cold || exit $?
head -8 "$OUT/trace5/run_kernel_stats.csv" | cut -c1-150
