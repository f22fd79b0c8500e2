#!/bin/bash
# Round 5, call F: end to end at the headline configuration: ranks 0, 3 and
# 7 of an 8-GPU cfg4 run, each rank's slice written as its own BAM (SEQ/QUAL, BAI) + VCF and run
# through the `svtrek audt` CLI on one GPU (tools/e2e_shard.py), then cfg4's contig 1 and the
# full cfg2 end to end.  One time limit per step; stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/r05_F
mkdir -p "$OUT"
export TMPDIR=/tmp
df -h /tmp > "$OUT/df.log" 2>&1
run() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] start $name" >> "$OUT/steps.log"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] end $name rc=$rc" >> "$OUT/steps.log"
  tail -4 "$OUT/$name.log" | cut -c1-600
  return $rc
}
run e2e_shard 800 python -u tools/e2e_shard.py --world 8 --ranks 0,3,7 -t 16 --reps 2 || exit $?
run e2e_c4 400 python -u tools/e2e_bench.py --workload cfg4_1m_delins_30x_hifi --region-sample 45455 -t 16 --reps 2 --inflate gpu || exit $?
