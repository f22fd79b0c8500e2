#!/bin/bash
# Round 5, call E: steps in flight (bench.py --inflight 2: two engine contexts / streams, step
# i + 1's index build beside step i's refine) against one, on cfg4, its emulated 8-GPU shards,
# cfg2 and cfg5.  One time limit per step; stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/r05_E
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_api.py tests/test_gpu_parity.py > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
b() { local n=$1; shift; timeout -k 10 400 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-cold "$@" \
  > "$OUT/$n.log" 2>&1 || { echo "$n failed"; tail -5 "$OUT/$n.log"; exit 1; }
  python3 - "$n" "$OUT/$n.log" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
ph = d["roofline"]["phases"]
print(f"{sys.argv[1]:>12}: step {d['ms_per_step']:.4f} ms (events {d['roofline']['step_ms_mean']:.4f})  index {ph['index_ms']:.4f}  refine {ph['refine_ms']:.4f}  {d['value']/1e6:.1f} M loci/s  verified {d['records_verified']}")
PY
}
b c4_k1 && b c4_k2 --inflight 2 && b c4_k1b && b c4_k2b --inflight 2 && \
b sh0_k1 --emulate-shard 8:0 && b sh0_k2 --emulate-shard 8:0 --inflight 2 && \
b sh3_k1 --emulate-shard 8:3 && b sh3_k2 --emulate-shard 8:3 --inflight 2 && \
b sh7_k1 --emulate-shard 8:7 && b sh7_k2 --emulate-shard 8:7 --inflight 2 && \
b c2_k1 --workload cfg2_10kdel_30x_ont && b c2_k2 --workload cfg2_10kdel_30x_ont --inflight 2 && \
b c5_k1 --workload cfg5_100k_60x_ul_ont --steps 10 && b c5_k2 --workload cfg5_100k_60x_ul_ont --steps 10 --inflight 2 || exit 1
