#!/bin/bash
# Round 5, call H: the single-pass lane index build (ix2_fused_kernel, svt_reindex) -- parity
# tests (reindex after load, several rebuilds), cfg4 bench lines against the two-kernel build
# (variants/x_nofused.so) at one and two steps in flight and on rank 3 of 8; then end to end on
# ranks 0, 3, 7 of an 8-GPU cfg4 run (tools/e2e_shard.py) and cfg4's contig-1 region.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/r05_H
mkdir -p "$OUT"
export TMPDIR=/tmp
W=cfg4_1m_delins_30x_hifi
bash tools/gpu_ab_pairs.sh r05_H_ab default\|$W\|--inflight\ 1 x_nofused\|$W\|--inflight\ 1 \
  default\|$W x_nofused\|$W default\|$W\|--emulate-shard\ 8:3 x_nofused\|$W\|--emulate-shard\ 8:3 \
  default\|$W\|--inflight\ 1 x_nofused\|$W\|--inflight\ 1 || exit $?
run() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] start $name" >> "$OUT/steps.log"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] end $name rc=$rc" >> "$OUT/steps.log"
  tail -4 "$OUT/$name.log" | cut -c1-600
  return $rc
}
run e2e_c4 300 python -u tools/e2e_bench.py --workload $W --region-sample 45455 -t 16 --reps 2 --inflate gpu || exit $?
run e2e_shard 600 python -u tools/e2e_shard.py --world 8 --ranks 0,3,7 -t 16 --reps 2 || exit $?
