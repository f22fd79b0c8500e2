#!/bin/bash
# Round 5, call AA: end to end with engine 0.23.4 (BGZF inflate 30 GB/s) -- the CLI's device
# batch size (256 MiB: ~5.8 K BGZF blocks, fewer than the 8 192 waves the inflate now keeps
# resident, vs 384 MiB) on cfg2 and cfg4's contig 1; in-tree engine vs variants/base (50a515f).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/r05_AA
mkdir -p "$OUT"
export TMPDIR=/tmp
summ() {
  python - "$1" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l)
        print(f"{d['workload'][:5]} {d['inflate']:>8} {d['engine']:>14}: {d['seconds_all']}  {(d['stages_last_run'] or '')[:140]}")
PY
}
timeout -k 10 800 python -u tools/e2e_bench.py --workload cfg2_10kdel_30x_ont --with-seq -t 16 --reps 3 \
  --inflate gpu,gpu:384 --libs tree,variants/base > "$OUT/e2e_c2.log" 2>&1 || { echo "e2e c2 failed"; tail -5 "$OUT/e2e_c2.log"; exit 1; }
summ "$OUT/e2e_c2.log"
timeout -k 10 500 python -u tools/e2e_bench.py --workload cfg4_1m_delins_30x_hifi --region-sample 45455 -t 16 --reps 3 \
  --inflate gpu,gpu:384 --libs tree,variants/base > "$OUT/e2e_c4.log" 2>&1 || { echo "e2e c4 failed"; tail -5 "$OUT/e2e_c4.log"; exit 1; }
summ "$OUT/e2e_c4.log"
echo done
