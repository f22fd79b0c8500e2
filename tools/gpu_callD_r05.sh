#!/bin/bash
# Round 5, call D: engine 0.22.1 (block-sum index scan: 3 launches per index build instead of 5):
# the parity / workload / API / BAM-decode tests, the cfg4 bench line, the emulated 8-GPU shards
# 0 / 3 / 7, cfg2, and a kernel trace of the cfg4 step.  One time limit per step; stops at the
# first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/r05_D
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_workloads.py tests/test_gpu_api.py tests/test_gpu_bam_decode.py \
  > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
b() { local n=$1; shift; timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-cold "$@" \
  > "$OUT/$n.log" 2>&1 || { echo "$n failed"; tail -5 "$OUT/$n.log"; exit 1; }
  python3 - "$n" "$OUT/$n.log" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
ph = d["roofline"]["phases"]
print(f"{sys.argv[1]:>12}: step {d['ms_per_step']:.4f} ms  index {ph['index_ms']:.4f}  refine {ph['refine_ms']:.4f}  {d['value']/1e6:.1f} M loci/s")
PY
}
b cfg4 && b sh0 --emulate-shard 8:0 && b sh3 --emulate-shard 8:3 && b sh7 --emulate-shard 8:7 && \
b cfg2 --workload cfg2_10kdel_30x_ont && b cfg4b || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
  python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-cold > "$OUT/trace.log" 2>&1 || { echo trace failed; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_sh3" -o run -- \
  python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-cold --emulate-shard 8:3 > "$OUT/trace_sh3.log" 2>&1 || { echo trace failed; exit 1; }
head -8 "$OUT/trace/run_kernel_stats.csv" | cut -c1-150
