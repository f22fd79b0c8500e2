#!/bin/bash
# Run ON THE GPU BOX: two SQ counter passes over the BGZF inflate bench (instruction mix and
# waits of inflate_kernel).   tools/gpu_infpmc.sh TAG
set -u
TAG=${1:?tag}
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
P1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES"
P2="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_WAVES"
i=0
for pass in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $pass --output-format csv -d "$OUT/p$i" -o run -- \
    python3 tools/bench_inflate.py --scale 0.1 --reps 1 > "$OUT/p$i.log" 2>&1 || { echo "fail p$i"; tail -5 "$OUT/p$i.log"; exit 1; }
done
echo "done"
