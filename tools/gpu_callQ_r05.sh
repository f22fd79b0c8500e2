#!/bin/bash
# Round 5, call Q: engine 0.23.1 + the match copy's ring and far loops apart (no flat loads):
# inflate GPU tests, the inflate kernel alone vs variants/base.so, SQ counters.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/${CALL_TAG:-r05_Q}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_inflate.py tests/test_gpu_bam_decode.py > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in new base; do
    lib=""; [ $v = base ] && lib=$PWD/variants/base.so
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
timeout -s KILL 200 rocprofv3 --pmc $P1 --output-format csv -d "$OUT/pmc_inf" -o run -- \
  python3 tools/bench_inflate.py --scale 0.1 --reps 1 > "$OUT/pmc_inf.log" 2>&1 || { echo "pmc failed"; exit 1; }
echo done
