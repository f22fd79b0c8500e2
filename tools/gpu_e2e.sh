#!/bin/bash
# Run ON THE GPU BOX: end-to-end CLI timings on BAMs with SEQ/QUAL (GPU vs CPU BGZF inflate):
# the CPU baseline's cfg4 region sample (1000 loci, 121 MB BAM), full cfg2 (10k loci, ~14 GB
# BAM, written first); then the inflate and POA benches.   tools/gpu_e2e.sh TAG
set -u
TAG=${1:?tag}
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] start $name" >> "$OUT/steps.log"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] end $name rc=$rc" >> "$OUT/steps.log"
  tail -2 "$OUT/$name.log" | cut -c1-400
  return $rc
}
df -h /tmp > "$OUT/df.log" 2>&1
run e2e_cfg4_region 300 python -u tools/e2e_bench.py --workload cfg4_1m_delins_30x_hifi --region-sample 1000 -t 16 --reps 3 || exit $?
run infbench 300 python tools/bench_inflate.py --scale 0.1 --reps 3 || exit $?
run poa 400 python tools/bench_poa.py --workload cfg3_50k_delins_30x_ont || exit $?
run e2e_cfg2_seq 900 python -u tools/e2e_bench.py --workload cfg2_10kdel_30x_ont --with-seq -t 16 --reps 2 || exit $?
