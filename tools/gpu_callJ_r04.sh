#!/bin/bash
# Round-4 closing run on engine 0.21.1: smoke, every GPU test, the default bench line and its
# kernel trace, then trace + PMC passes of cfg4, cfg5, cfg3 and cfg2 (traffic.json).  Stops at
# the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
bash tools/gpu_full.sh r04_J --no-cfg5 && \
bash tools/gpu_profile.sh r04J_cfg4 --workload cfg4_1m_delins_30x_hifi && \
bash tools/gpu_profile.sh r04J_cfg5 --workload cfg5_100k_60x_ul_ont && \
bash tools/gpu_profile.sh r04J_cfg3 --workload cfg3_50k_delins_30x_ont && \
bash tools/gpu_profile.sh r04J_cfg2 --workload cfg2_10kdel_30x_ont
