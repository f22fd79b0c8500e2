#!/bin/bash
# Round 5, call G: the vector-state BGZF literal loop (SVT_IW_VEC, default) against the scalar
# one (variants_inf/i_novec.so): zlib identity + device BAM decode tests, tools/bench_inflate.py
# on both, SQ counters of the new one, then cfg2 end to end (device inflate + decode).  Then the
# refine's phase-2 changes (odd-even merge sort, prefilled band rows, l0 counted on registers):
# parity tests, and cfg4 bench lines of the default against variants/r_*.so.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/r05_G
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_inflate.py tests/test_gpu_bam_decode.py tests/test_gpu_cli.py tests/test_gpu_parity.py \
  tests/test_gpu_workloads.py > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
for v in default i_novec default i_novec; do
  lib=$PWD/svtrek_amd/libsvtrek_hip.so; [ $v != default ] && lib=$PWD/variants_inf/$v.so
  SVTREK_ENGINE_LIB=$lib timeout -k 10 300 python tools/bench_inflate.py --scale 0.1 --reps 3 > "$OUT/inf_$v.log" 2>&1 \
    || { echo "bench $v failed"; tail -5 "$OUT/inf_$v.log"; exit 1; }
  echo "$v $(tail -1 "$OUT/inf_$v.log" | cut -c1-330)"
done
P1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_BUSY_CYCLES"
timeout -s KILL 200 rocprofv3 --pmc $P1 --output-format csv -d "$OUT/pmc1" -o run -- \
  python3 tools/bench_inflate.py --scale 0.1 --reps 1 > "$OUT/pmc1.log" 2>&1 || { echo "pmc failed"; exit 1; }
timeout -k 10 600 python -u tools/e2e_bench.py --workload cfg2_10kdel_30x_ont --with-seq -t 16 --reps 2 --inflate gpu \
  > "$OUT/e2e_cfg2.log" 2>&1 || { echo "e2e failed"; tail -5 "$OUT/e2e_cfg2.log"; exit 1; }
tail -1 "$OUT/e2e_cfg2.log" | cut -c1-500
NO_TESTS=1 bash tools/gpu_ab_pairs.sh r05_G_ab default\|cfg4_1m_delins_30x_hifi\|--inflight\ 1 \
  r_none\|cfg4_1m_delins_30x_hifi\|--inflight\ 1 r_bitonic\|cfg4_1m_delins_30x_hifi\|--inflight\ 1 \
  r_noprefill\|cfg4_1m_delins_30x_hifi\|--inflight\ 1 r_nol0\|cfg4_1m_delins_30x_hifi\|--inflight\ 1 \
  r_diag8\|cfg4_1m_delins_30x_hifi\|--inflight\ 1\ --no-verify default\|cfg4_1m_delins_30x_hifi\|--inflight\ 1 \
  r_none\|cfg4_1m_delins_30x_hifi\|--inflight\ 1 default\|cfg4_1m_delins_30x_hifi || exit $?
