#!/bin/bash
# Round 5, call AJ: the tree on a fresh box -- the whole -m gpu suite, smoke(), then census / emit
# groups per wave (SVT_IX2_GPW 1 = in-tree, 2, 4) on cfg4 and rank 3 of 8, alternating, then the
# default bench line (three steps in flight, with its CPU baseline) and a kernel trace of it.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/r05_AJ
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests \
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
  for v in gpw1 gpw2 gpw4; do
    lib=""; [ $v != gpw1 ] && lib=$PWD/variants/$v.so
    for args in "" "--emulate-shard 8:3"; do
      tag="${v}_$(echo "$args" | tr -c 'a-z0-9' '_')_$rep"
      SVTREK_ENGINE_LIB=$lib timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-cold $args \
        > "$OUT/$tag.log" 2>&1 || { echo "$tag failed"; tail -5 "$OUT/$tag.log"; exit 1; }
      line "$tag" "$OUT/$tag.log"
    done
  done
done
timeout -k 10 300 python bench.py > "$OUT/bench.log" 2>&1 || { tail -5 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log" | cut -c1-300
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
  python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-cold > "$OUT/bench_trace.log" 2>&1 || { tail -5 "$OUT/bench_trace.log"; exit 1; }
echo done
