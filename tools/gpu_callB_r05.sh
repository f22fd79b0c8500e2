#!/bin/bash
# Round 5, call B: parity of engine 0.22.0 (buffer-descriptor span walk, band-size min_count),
# then cfg4 bench lines of the A/B variants (variants/*.so: the 0.21 walk, buffer walk only,
# both, the phase-0 / phase-0+1 diagnostic builds) and one SQ counter pass of the old and new
# lane kernel.  One time limit per step; stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/r05_B
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_workloads.py tests/test_gpu_api.py > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
SVTREK_ENGINE_LIB=$PWD/variants/v7_flat.so timeout -k 10 400 python -u -m pytest -x -q --timeout 240 \
  --timeout-method thread -m gpu tests/test_gpu_parity.py > "$OUT/pytest_flat.log" 2>&1
rc=$?; tail -2 "$OUT/pytest_flat.log"; [ $rc -eq 0 ] || exit $rc
NO_TESTS=1 bash tools/gpu_ab_pairs.sh r05_B_ab default\|cfg4_1m_delins_30x_hifi \
  v0_old\|cfg4_1m_delins_30x_hifi \
  v1_buf\|cfg4_1m_delins_30x_hifi \
  v2_novl\|cfg4_1m_delins_30x_hifi \
  v3_diag6\|cfg4_1m_delins_30x_hifi\|--no-verify \
  v4_diag8\|cfg4_1m_delins_30x_hifi\|--no-verify \
  v6_diag8_novl\|cfg4_1m_delins_30x_hifi\|--no-verify \
  v7_flat\|cfg4_1m_delins_30x_hifi \
  default\|cfg4_1m_delins_30x_hifi \
  v0_old\|cfg4_1m_delins_30x_hifi \
  v2_novl\|cfg4_1m_delins_30x_hifi || exit $?
timeout -k 10 120 rocprofv3 -L > "$OUT/counters_avail.txt" 2>&1 || true
EXTRA=""
for c in SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC; do
  grep -qw "$c" "$OUT/counters_avail.txt" && EXTRA="$EXTRA $c"
done
echo "extra counters:$EXTRA"
for v in v0_old default; do
  lib=$PWD/svtrek_amd/libsvtrek_hip.so; [ $v != default ] && lib=$PWD/variants/$v.so
  SVTREK_ENGINE_LIB=$lib timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
    SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d "$OUT/sq_$v" -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-cold > "$OUT/sq_$v.log" 2>&1 || { echo "sq $v failed"; exit 1; }
  if [ -n "$EXTRA" ]; then
    SVTREK_ENGINE_LIB=$lib timeout -s KILL 200 rocprofv3 --pmc $EXTRA --output-format csv -d "$OUT/sq2_$v" -o run -- \
      python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-cold > "$OUT/sq2_$v.log" 2>&1 || { echo "sq2 $v failed"; exit 1; }
  fi
done
for k in refine_lane_kernel refine_redo_kernel ix2_census_kernel ix2_emit_kernel; do echo "== $k"; python3 tools/pmc_summary.py $k "$OUT"/sq_v0_old "$OUT"/sq_default "$OUT"/sq2_v0_old "$OUT"/sq2_default; done > "$OUT/sq_summary.txt" 2>&1 || true
cat "$OUT/sq_summary.txt" | head -40
