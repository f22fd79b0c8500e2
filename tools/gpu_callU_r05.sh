#!/bin/bash
# Round 5, call U: engine 0.23.2 on a fresh box -- the whole -m gpu suite, smoke(), the default
# bench line, rank slices 0/3/7 of the 8-GPU split, end to end on cfg2 and cfg4's contig 1 (vs
# variants/base = HEAD 50a515f), and the inflate kernel alone.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/r05_U
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 560 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests \
  > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -5 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 300 python bench.py > "$OUT/bench.log" 2>&1 || { tail -5 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log" | cut -c1-300
for r in 0 3 7; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-cold --emulate-shard 8:$r \
    > "$OUT/shard_$r.log" 2>&1 || { echo "shard $r failed"; tail -5 "$OUT/shard_$r.log"; exit 1; }
  python - "$r" "$OUT/shard_$r.log" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(f"rank {sys.argv[1]} of 8: {d['ms_per_step']:.4f} ms per step")
PY
done
timeout -k 10 300 python tools/bench_inflate.py --scale 0.1 --reps 3 > "$OUT/inf.log" 2>&1 || { echo "inf failed"; exit 1; }
tail -1 "$OUT/inf.log" | cut -c1-330
summ() {
  python - "$1" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l)
        print(f"{d['workload'][:5]} {d['engine']:>14}: {d['seconds_all']}  {(d['stages_last_run'] or '')[:150]}")
PY
}
timeout -k 10 600 python -u tools/e2e_bench.py --workload cfg2_10kdel_30x_ont --with-seq -t 16 --reps 3 --inflate gpu \
  --libs tree,variants/base > "$OUT/e2e_c2.log" 2>&1 || { echo "e2e c2 failed"; tail -5 "$OUT/e2e_c2.log"; exit 1; }
summ "$OUT/e2e_c2.log"
timeout -k 10 400 python -u tools/e2e_bench.py --workload cfg4_1m_delins_30x_hifi --region-sample 45455 -t 16 --reps 3 \
  --inflate gpu --libs tree,variants/base > "$OUT/e2e_c4.log" 2>&1 || { echo "e2e c4 failed"; tail -5 "$OUT/e2e_c4.log"; exit 1; }
summ "$OUT/e2e_c4.log"
echo done
