#!/bin/bash
# Run ON THE GPU BOX: the other BASELINE workloads (the headline cfg4 line is bench.py's
# default) and the per-rank work of the 8-GPU run, one time limit per step; stops at the
# first failure.   tools/gpu_configs.sh TAG
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
  tail -1 "$OUT/$name.log" | cut -c1-400
}
if [ -z "${CONFIGS_ONLY:-}" ]; then   # CONFIGS_ONLY=1: the BASELINE workloads only
run cfg4_shard8_r0 300 --emulate-shard 8:0 --steps 20 --warmup 3 --no-cpu-baseline
run cfg4_shard8_r7 300 --emulate-shard 8:7 --steps 20 --warmup 3 --no-cpu-baseline
run cfg4_scale0125 300 --scale 0.125 --steps 20 --warmup 3 --no-cpu-baseline
fi
run cfg3 300 --workload cfg3_50k_delins_30x_ont --steps 20 --warmup 3 --no-cpu-baseline
run cfg2 300 --workload cfg2_10kdel_30x_ont --steps 20 --warmup 3 --no-cpu-baseline
run cfg1 200 --workload cfg1_100del_10x --steps 20 --warmup 3 --no-cpu-baseline
run cfg5 900 --workload cfg5_100k_60x_ul_ont --steps 10 --warmup 2 --no-cpu-baseline
