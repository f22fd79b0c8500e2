#!/bin/bash
# Round 5, call S/T: BGZF inflate loop shapes against variants (see the NOTE of the run).
# everything off the fast path) vs variants/flat3.so (up to three literals an iteration, no inner
# loop) vs variants/base.so (HEAD 50a515f); inflate / BAM-decode GPU tests on the in-tree build,
# SQ counters of each.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/${CALL_TAG:-r05_S}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_inflate.py tests/test_gpu_bam_decode.py > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in new single base; do
    lib=""; [ $v != new ] && lib=$PWD/variants/$v.so
    SVTREK_ENGINE_LIB=$lib timeout -k 10 300 python tools/bench_inflate.py --scale 0.1 --reps 3 > "$OUT/inf_${v}_$rep.log" 2>&1 \
      || { echo "inf $v failed"; tail -5 "$OUT/inf_${v}_$rep.log"; exit 1; }
    python - "$v $rep" "$OUT/inf_${v}_$rep.log" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(sys.argv[1], d["kernel_ms"], "ms", d["kernel_gbs"], "GB/s identical", d["identical_to_zlib"])
PY
  done
done
P1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_WAIT_ANY"
for v in new single; do
  lib=""; [ $v != new ] && lib=$PWD/variants/$v.so
  SVTREK_ENGINE_LIB=$lib timeout -s KILL 200 rocprofv3 --pmc $P1 --output-format csv -d "$OUT/pmc_$v" -o run -- \
    python3 tools/bench_inflate.py --scale 0.1 --reps 1 > "$OUT/pmc_$v.log" 2>&1 || { echo "pmc failed"; exit 1; }
done
echo done
