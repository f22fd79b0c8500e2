#!/bin/bash
# Run ON THE GPU BOX: SQ / SQC counter passes over the BGZF inflate bench (instruction mix, waits,
# scalar-cache behaviour of inflate_kernel).   tools/gpu_infpmc.sh TAG [ENGINE_LIB]
set -u
TAG=${1:?tag}
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
[ -n "${2:-}" ] && export SVTREK_ENGINE_LIB=$2
P1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_BUSY_CYCLES"
P2="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAVES SQ_ACTIVE_INST_SCA"
P3="SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_DCACHE_REQ SQC_ICACHE_MISSES GRBM_GUI_ACTIVE"
P4="SQ_INST_CYCLES_SALU SQ_INSTS_SMEM_NORM SQ_WAIT_ANY SQ_IFETCH"
i=0
for pass in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $pass --output-format csv -d "$OUT/p$i" -o run -- \
    python3 tools/bench_inflate.py --scale 0.1 --reps 1 > "$OUT/p$i.log" 2>&1 || { echo "fail p$i"; tail -5 "$OUT/p$i.log"; }
done
python3 - "$OUT" <<'PY'
import csv, collections, sys, os
out = sys.argv[1]
for p in sorted(os.listdir(out)):
    f = os.path.join(out, p, "run_counter_collection.csv")
    if not os.path.exists(f):
        continue
    agg, disp = collections.defaultdict(float), set()
    for r in csv.DictReader(open(f)):
        if "inflate_kernel" in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            disp.add(r["Dispatch_Id"])
    print(p, len(disp), {k: f"{v / max(len(disp), 1):.4g}" for k, v in agg.items()})
PY
