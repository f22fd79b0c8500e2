#!/bin/bash
# Round 5, call L: the stream walk's range count (32 768 ranges of <= 65 536 ops by default now)
# on cfg2 / cfg3 / cfg5 against 131 072 (SVTREK_IX_RANGES); then the device BAM decode's batch
# buffers pinned (SVTREK_DEC_PINNED=1) with the feed in 1 or 4 parts, end to end on cfg2 and
# cfg4's contig 1.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/r05_L
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_workloads.py > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
line() {  # tag log
  python - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
ph = d["roofline"]["phases"]
print(f"{sys.argv[1]:>40}: step {d['ms_per_step']:.4f} ms  index {ph['index_ms']:.4f}  refine {ph['refine_ms']:.4f}")
PY
}
for spec in cfg2_10kdel_30x_ont:default cfg2_10kdel_30x_ont:131072 cfg2_10kdel_30x_ont:16384 \
            cfg3_50k_delins_30x_ont:default cfg3_50k_delins_30x_ont:131072 \
            cfg5_100k_60x_ul_ont:default cfg5_100k_60x_ul_ont:131072; do
  wl=${spec%%:*}; nr=${spec#*:}
  if [ "$nr" = default ]; then unset SVTREK_IX_RANGES; else export SVTREK_IX_RANGES=$nr; fi
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-cold --workload $wl --inflight 1 \
    > "$OUT/${wl}_$nr.log" 2>&1 || { echo "$spec failed"; tail -5 "$OUT/${wl}_$nr.log"; exit 1; }
  line "$spec" "$OUT/${wl}_$nr.log"
done
unset SVTREK_IX_RANGES
e2e() {  # name, libdir ("" = in-tree), pinned, workload args...
  local name=$1 lib=$2 pin=$3; shift 3
  LD_LIBRARY_PATH=${lib:+$PWD/$lib} SVTREK_DEC_PINNED=$pin timeout -k 10 400 python -u tools/e2e_bench.py "$@" -t 16 --reps 2 \
    --inflate gpu > "$OUT/e2e_$name.log" 2>&1 || { echo "e2e $name failed"; tail -5 "$OUT/e2e_$name.log"; return 1; }
  python - "$name" "$OUT/e2e_$name.log" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(f"{sys.argv[1]:>14}: {d['seconds_all']}  {d['stages_last_run'][:160]}")
PY
}
e2e c2_pin_p4 variants/p4 1 --workload cfg2_10kdel_30x_ont --with-seq || exit 1
e2e c2_pin_p1 "" 1 --workload cfg2_10kdel_30x_ont --with-seq || exit 1
e2e c2_page_p1 "" 0 --workload cfg2_10kdel_30x_ont --with-seq || exit 1
e2e c4_pin_p4 variants/p4 1 --workload cfg4_1m_delins_30x_hifi --region-sample 45455 || exit 1
e2e c4_page_p1 "" 0 --workload cfg4_1m_delins_30x_hifi --region-sample 45455 || exit 1
