#!/bin/bash
# Run ON THE GPU BOX: the headline bench (cfg2, with CPU baseline) and the other BASELINE
# workloads (kernel throughput only).  Each step has its own time limit; stops at the first failure.
set -u
TAG=${1:?tag}
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/cfg_$TAG
mkdir -p "$OUT"
run() {  # name, timeout, args...
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] $name" >> "$OUT/steps.log"
  timeout -k 10 "$t" python -u bench.py "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" >> "$OUT/steps.log"
  [ $rc -eq 0 ] || { tail -20 "$OUT/$name.log"; exit $rc; }
  tail -1 "$OUT/$name.log"
}
[ "${SKIP_CFG2:-0}" = 1 ] || run cfg2 400 --steps 20 --warmup 3
run cfg4 400 --workload cfg4_1m_delins_30x_hifi --steps 10 --warmup 2 --no-cpu-baseline
run cfg3 600 --workload cfg3_50k_delins_30x_ont --steps 10 --warmup 2 --no-cpu-baseline
#run cfg5q 900 --workload cfg5_100k_60x_ul_ont --scale 0.25 --steps 10 --warmup 2 --no-cpu-baseline
