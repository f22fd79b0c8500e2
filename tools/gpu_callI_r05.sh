#!/bin/bash
# Round 5, call I: the single-pass lane index build in workgroup order (no ticket atomics) --
# parity / api (graph replay) / inflate / BAM decode tests, cfg4 bench lines against the
# two-pass build (variants/x_nofused.so); refine_lane_kernel's phase attribution
# (variants/x_phase.so); then the overlapped feed (BAM bytes in 4 parts, part k inflating while
# k + 1 crosses PCIe) against one part (variants/p1) on cfg2 end to end.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/r05_I
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_api.py tests/test_gpu_parity.py tests/test_gpu_inflate.py tests/test_gpu_bam_decode.py \
  > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
W=cfg4_1m_delins_30x_hifi
NO_TESTS=1 bash tools/gpu_ab_pairs.sh r05_I_ab default\|$W\|--inflight\ 1 x_nofused\|$W\|--inflight\ 1 \
  default\|$W x_nofused\|$W default\|$W\|--emulate-shard\ 8:3 x_nofused\|$W\|--emulate-shard\ 8:3 \
  default\|$W\|--inflight\ 1 || exit $?
SVTREK_ENGINE_LIB=$PWD/variants/x_phase.so timeout -k 10 200 python tools/phase_prof.py --workload $W \
  > "$OUT/phase.log" 2>&1 || { echo "phase failed"; tail -5 "$OUT/phase.log"; exit 1; }
tail -1 "$OUT/phase.log"
timeout -k 10 400 python -u tools/e2e_bench.py --workload cfg2_10kdel_30x_ont --with-seq -t 16 --reps 2 --inflate gpu \
  > "$OUT/e2e_cfg2.log" 2>&1 || { echo "e2e failed"; tail -5 "$OUT/e2e_cfg2.log"; exit 1; }
tail -1 "$OUT/e2e_cfg2.log" | cut -c1-700
LD_LIBRARY_PATH=$PWD/variants/p1 timeout -k 10 400 python -u tools/e2e_bench.py --workload cfg2_10kdel_30x_ont --with-seq \
  -t 16 --reps 2 --inflate gpu > "$OUT/e2e_cfg2_p1.log" 2>&1 || { echo "e2e p1 failed"; tail -5 "$OUT/e2e_cfg2_p1.log"; exit 1; }
tail -1 "$OUT/e2e_cfg2_p1.log" | cut -c1-700
