#!/bin/bash
# Round 5, call K: phase 1's slot stream (lane_stream: windows of 65-512 events walked as one
# stream of 64-event slots, 4 in flight across windows) -- parity / workload / api tests, cfg4
# and rank-3-of-8 bench lines against lane_walk per window (variants/x_nostream.so) and other
# stream caps, and the new phase attribution.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/r05_K
mkdir -p "$OUT"
export TMPDIR=/tmp
W=cfg4_1m_delins_30x_hifi
bash tools/gpu_ab_pairs.sh r05_K_ab default\|$W\|--inflight\ 1 x_nostream\|$W\|--inflight\ 1 \
  x_smax256\|$W\|--inflight\ 1 x_smax1024\|$W\|--inflight\ 1 default\|$W x_nostream\|$W \
  default\|$W\|--emulate-shard\ 8:3 x_nostream\|$W\|--emulate-shard\ 8:3 default\|$W\|--inflight\ 1 \
  x_nostream\|$W\|--inflight\ 1 || exit $?
SVTREK_ENGINE_LIB=$PWD/variants/x_phase.so timeout -k 10 200 python tools/phase_prof.py --workload $W \
  > "$OUT/phase.log" 2>&1 || { echo "phase failed"; tail -5 "$OUT/phase.log"; exit 1; }
tail -1 "$OUT/phase.log"
