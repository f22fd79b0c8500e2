#!/bin/bash
# Round-4 A/B: the stream walk's prefetch depth (SVT_IX_PF=2) at 7 and 8 waves per SIMD against
# the default (PF=3, 7 waves), on the three stream-walk BASELINE workloads.  No tests (bench only:
# the variants change occupancy knobs, not the algorithm; the winner is re-tested as the default).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
NO_TESTS=1 bash tools/gpu_ab_pairs.sh r04_pf \
  "default|cfg5_100k_60x_ul_ont" "p2w7|cfg5_100k_60x_ul_ont" "p2w8|cfg5_100k_60x_ul_ont" \
  "default|cfg3_50k_delins_30x_ont" "p2w7|cfg3_50k_delins_30x_ont" "p2w8|cfg3_50k_delins_30x_ont" \
  "default|cfg2_10kdel_30x_ont" "p2w7|cfg2_10kdel_30x_ont" "p2w8|cfg2_10kdel_30x_ont" \
  "default|cfg5_100k_60x_ul_ont"
