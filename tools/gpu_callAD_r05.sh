#!/bin/bash
# Round 5, call AD: end to end with engine 0.23.4, the CLI's device batch buffers pageable (the
# default) vs pinned (SVTREK_DEC_PINNED=1), now that the feed overlaps a batch's copy with the
# previous batch's inflate; cfg2 and cfg4's contig 1.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/r05_AD
mkdir -p "$OUT"
export TMPDIR=/tmp
mkdir -p /tmp/e2e_c2 /tmp/e2e_c4
summ() {
  python - "$1" "$2" <<'PY'
import json, sys
for l in open(sys.argv[2]):
    if l.startswith("{"):
        d = json.loads(l)
        print(f"{sys.argv[1]:>6} {d['workload'][:5]}: {d['seconds_all']}  {(d['stages_last_run'] or '')[:150]}")
PY
}
for pin in 0 1; do
  SVTREK_DEC_PINNED=$pin timeout -k 10 600 python -u tools/e2e_bench.py --workload cfg2_10kdel_30x_ont --with-seq -t 16 --reps 3 \
    --inflate gpu --dir /tmp/e2e_c2 > "$OUT/e2e_c2_pin$pin.log" 2>&1 || { echo "e2e c2 failed"; tail -5 "$OUT/e2e_c2_pin$pin.log"; exit 1; }
  summ "pin$pin" "$OUT/e2e_c2_pin$pin.log"
done
for pin in 0 1; do
  SVTREK_DEC_PINNED=$pin timeout -k 10 400 python -u tools/e2e_bench.py --workload cfg4_1m_delins_30x_hifi --region-sample 45455 -t 16 \
    --reps 3 --inflate gpu --dir /tmp/e2e_c4 > "$OUT/e2e_c4_pin$pin.log" 2>&1 || { echo "e2e c4 failed"; tail -5 "$OUT/e2e_c4_pin$pin.log"; exit 1; }
  summ "pin$pin" "$OUT/e2e_c4_pin$pin.log"
done
timeout -k 10 700 python -u tools/e2e_shard.py --world 8 --ranks 0,3,7 -t 16 --reps 2 > "$OUT/e2e_shard.log" 2>&1 \
  || { echo "e2e shard failed"; tail -5 "$OUT/e2e_shard.log"; exit 1; }
tail -4 "$OUT/e2e_shard.log" | cut -c1-600
echo done
