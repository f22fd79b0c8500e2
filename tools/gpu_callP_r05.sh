#!/bin/bash
# Round 5, call P: engine 0.23.1 -- the BGZF inflate's match path on the vector side (length /
# distance decode, checks and copy on the lane copies; only branches on the scalar unit).  The
# inflate / BAM-decode / CLI GPU tests, the inflate kernel alone against variants/base.so, SQ
# counters of one launch, then end to end on cfg2 and cfg4's contig 1 against variants/base.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/r05_P
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_inflate.py tests/test_gpu_bam_decode.py tests/test_gpu_cli.py > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in new base; do
    lib=""; [ $v = base ] && lib=$PWD/variants/base.so
    SVTREK_ENGINE_LIB=$lib timeout -k 10 300 python tools/bench_inflate.py --scale 0.1 --reps 3 > "$OUT/inf_${v}_$rep.log" 2>&1 \
      || { echo "inf $v failed"; tail -5 "$OUT/inf_${v}_$rep.log"; exit 1; }
    echo "$v $rep: $(tail -1 "$OUT/inf_${v}_$rep.log" | cut -c1-330)"
  done
done
P1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_WAIT_ANY"
timeout -s KILL 200 rocprofv3 --pmc $P1 --output-format csv -d "$OUT/pmc_inf" -o run -- \
  python3 tools/bench_inflate.py --scale 0.1 --reps 1 > "$OUT/pmc_inf.log" 2>&1 || { echo "pmc failed"; exit 1; }
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
