#!/bin/bash
# Round 5, call O (its BAM-decode / inflate / CLI tests passed in a first run: 28 green): svt_bam_dec_feed pipelined one batch deep (a batch's H2D copy beside the
# previous batch's inflate) -- the BAM-decode / inflate / CLI GPU tests, then end to end on cfg2
# (13.8 GB BAM with SEQ/QUAL) and cfg4's contig 1, in-tree engine vs variants/base (HEAD 50a515f),
# alternating reps on the same files.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/r05_O
mkdir -p "$OUT"
export TMPDIR=/tmp
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

# where the inflate kernel's time goes: per-block counts / ticks of the -DSVT_PHASE_PROF=1 build
SVTREK_ENGINE_LIB=$PWD/variants/x_iprof.so timeout -k 10 300 python tools/bench_inflate.py --scale 0.1 --reps 2 --phase \
  > "$OUT/inf_prof.log" 2>&1 || { echo "prof failed"; tail -5 "$OUT/inf_prof.log"; exit 1; }
tail -1 "$OUT/inf_prof.log" | cut -c1-900
timeout -k 10 300 python tools/bench_inflate.py --scale 0.1 --reps 3 > "$OUT/inf.log" 2>&1 || { echo "inf failed"; exit 1; }
tail -1 "$OUT/inf.log" | cut -c1-400
echo done
