#!/bin/bash
# Round 5, call AE: the lane build's emit walking the group's stretch from LDS (LDS-DMA copy,
# SVT_IX2_SCAP) -- index parity / workload GPU tests on the in-tree build, then cfg4 and rank-3
# bench lines of the variants (s0 = walk from HBM as 0.23.4), alternating, then FETCH_SIZE of the
# emit for s0 and s576.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/r05_AE
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_workloads.py > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
line() {  # tag log
  python - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
ph = d["roofline"]["phases"]
print(f"{sys.argv[1]:>28}: step {d['ms_per_step']:.4f} ms  index {ph['index_ms']:.4f}  refine {ph['refine_ms']:.4f}")
PY
}
for rep in 1 2; do
  for v in s0 s576 s576e192 s512e192 s576w1; do
    for args in "" "--emulate-shard 8:3"; do
      tag="${v}_$(echo "$args" | tr -c 'a-z0-9' '_')_$rep"
      SVTREK_ENGINE_LIB=$PWD/variants/$v.so timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-cold $args \
        > "$OUT/$tag.log" 2>&1 || { echo "$tag failed"; tail -5 "$OUT/$tag.log"; exit 1; }
      line "$tag" "$OUT/$tag.log"
    done
  done
done
for v in s0 s576; do
  SVTREK_ENGINE_LIB=$PWD/variants/$v.so timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE WRITE_SIZE --output-format csv -d "$OUT/pmc_$v" -o run -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-cold --inflight 1 > "$OUT/pmc_$v.log" 2>&1 || { echo "pmc $v failed"; exit 1; }
done
echo done
