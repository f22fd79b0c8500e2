#!/bin/bash
# Round-4 A/B: phase 1 of the lane kernel packing windows of <= 64 events into shared slots
# (SVT_PACK=1, the default build) against one window per walk (variants/nopack.so), after the
# parity / workload GPU tests on the packed default.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
bash tools/gpu_ab_pairs.sh r04_pack \
  "default|cfg4_1m_delins_30x_hifi" "nopack|cfg4_1m_delins_30x_hifi" "default|cfg4_1m_delins_30x_hifi" "nopack|cfg4_1m_delins_30x_hifi" \
  "default|cfg4_1m_delins_30x_hifi|--emulate-shard 8:3" "nopack|cfg4_1m_delins_30x_hifi|--emulate-shard 8:3" \
  "default|cfg5_100k_60x_ul_ont" "nopack|cfg5_100k_60x_ul_ont"
