#!/bin/bash
# Round 5, call N: engine 0.23.0 (lane_walk fed by v_readlane, branch-free member stores) --
# the whole -m gpu suite, smoke(), then cfg4 / rank-3 bench lines against variants/base.so
# (HEAD 50a515f's engine), alternating, and the default bench line with its CPU baseline.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/${CALL_TAG:-r05_N}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 560 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests \
  > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -5 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
line() {  # tag log
  python - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
ph = d["roofline"]["phases"]
print(f"{sys.argv[1]:>28}: step {d['ms_per_step']:.4f} ms  index {ph['index_ms']:.4f}  refine {ph['refine_ms']:.4f}")
PY
}
for rep in 1 2; do
  for v in new base; do
    lib=""; [ $v = base ] && lib=$PWD/variants/base.so
    for args in "--inflight 1" "" "--emulate-shard 8:3"; do
      tag="${v}_$(echo "$args" | tr -c 'a-z0-9' '_')_$rep"
      SVTREK_ENGINE_LIB=$lib timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-cold $args \
        > "$OUT/$tag.log" 2>&1 || { echo "$tag failed"; tail -5 "$OUT/$tag.log"; exit 1; }
      line "$tag" "$OUT/$tag.log"
    done
  done
done
timeout -k 10 300 python bench.py > "$OUT/bench.log" 2>&1 || { tail -5 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log" | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
  python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-cold > "$OUT/bench_trace.log" 2>&1 || { tail -5 "$OUT/bench_trace.log"; exit 1; }
P1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_WAIT_ANY"
timeout -s KILL 200 rocprofv3 --pmc $P1 --output-format csv -d "$OUT/pmc_sq" -o run -- \
  python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-cold --inflight 1 > "$OUT/pmc_sq.log" 2>&1 || { echo "pmc failed"; exit 1; }
echo done
