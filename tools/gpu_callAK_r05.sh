#!/bin/bash
# Round 5, call AK: where the cfg4 emit's extra HBM reads come from -- the index build alone
# (tools/ix_only.py: load + 5 rebuilds, no refine) on the in-tree engine and on a diagnostic build
# whose emit skips the per-lane CIGAR walk (-DSVT_DIAG=23: no stream reads; offsets and event rows
# still written), each with a kernel trace and the RDREQ / WRITE_SIZE PMC passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/r05_AK
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in tree diag23; do
  lib=""; [ $v != tree ] && lib=$PWD/variants/$v.so
  SVTREK_ENGINE_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${v}_trace" -o run -- \
    python3 tools/ix_only.py > "$OUT/${v}_trace.log" 2>&1 || { echo "$v trace failed"; tail -5 "$OUT/${v}_trace.log"; exit 1; }
  SVTREK_ENGINE_LIB=$lib timeout -s KILL 200 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum \
    --output-format csv -d "$OUT/${v}_rdreq" -o run -- python3 tools/ix_only.py > "$OUT/${v}_rdreq.log" 2>&1 || { echo "$v rdreq failed"; exit 1; }
  SVTREK_ENGINE_LIB=$lib timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE \
    --output-format csv -d "$OUT/${v}_write" -o run -- python3 tools/ix_only.py > "$OUT/${v}_write.log" 2>&1 || { echo "$v write failed"; exit 1; }
  echo "$v ok"
done
echo done
