#!/bin/bash
# Round 5, call C: the multi-literal BGZF inflate (SVT_IW_MULTI; root tables of 10 / 11 / 12 bits):
# zlib identity and device BAM decode tests on the default build and the variants, then
# tools/bench_inflate.py on each (variants_inf/*.so; i0_single = the round-4 decoder), then the
# SQ counters of the default.  One time limit per step; stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/r05_C
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_inflate.py tests/test_gpu_bam_decode.py > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
for v in i11 i12; do
  SVTREK_ENGINE_LIB=$PWD/variants_inf/$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 240 \
    --timeout-method thread -m gpu tests/test_gpu_inflate.py > "$OUT/pytest_$v.log" 2>&1
  rc=$?; tail -1 "$OUT/pytest_$v.log"; [ $rc -eq 0 ] || exit $rc
done
for v in default i0_single i11 i12 default; do
  lib=$PWD/svtrek_amd/libsvtrek_hip.so; [ $v != default ] && lib=$PWD/variants_inf/$v.so
  SVTREK_ENGINE_LIB=$lib timeout -k 10 300 python tools/bench_inflate.py --scale 0.1 --reps 3 > "$OUT/inf_$v.log" 2>&1 \
    || { echo "bench $v failed"; tail -5 "$OUT/inf_$v.log"; exit 1; }
  echo "$v $(tail -1 "$OUT/inf_$v.log" | cut -c1-400)"
done
P1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_BUSY_CYCLES"
timeout -s KILL 200 rocprofv3 --pmc $P1 --output-format csv -d "$OUT/pmc1" -o run -- \
  python3 tools/bench_inflate.py --scale 0.1 --reps 1 > "$OUT/pmc1.log" 2>&1 || { echo "pmc failed"; exit 1; }
echo done
