#!/bin/bash
# Round-4 closing run on engine 0.21 (2/2): trace + PMC passes of the long-read BASELINE
# workloads, the 8-GPU run's per-rank slices, and an A/B of ix_copy_kernel held to 7 waves per
# SIMD (variants/copy7.so) against its natural 5, and of the lane kernel's long-span walk
# with 2 slots in flight (variants/lwu2.so) against 4.  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
bash tools/gpu_profile.sh r04I_cfg5 --workload cfg5_100k_60x_ul_ont && \
bash tools/gpu_profile.sh r04I_cfg3 --workload cfg3_50k_delins_30x_ont && \
bash tools/gpu_profile.sh r04I_cfg2 --workload cfg2_10kdel_30x_ont && \
bash tools/gpu_profile.sh r04I_cfg1 --workload cfg1_100del_10x && \
B='python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-cold' && \
bash tools/gpu_steps.sh r04I_sh "r0|200|$B --emulate-shard 8:0" "r3|200|$B --emulate-shard 8:3" "r7|200|$B --emulate-shard 8:7" && \
NO_TESTS=1 bash tools/gpu_ab_pairs.sh r04_copy \
  "default|cfg2_10kdel_30x_ont" "copy7|cfg2_10kdel_30x_ont" "default|cfg3_50k_delins_30x_ont" "copy7|cfg3_50k_delins_30x_ont" \
  "default|cfg2_10kdel_30x_ont" "copy7|cfg2_10kdel_30x_ont" && \
NO_TESTS=1 bash tools/gpu_ab_pairs.sh r04_lwu \
  "default|cfg4_1m_delins_30x_hifi" "lwu2|cfg4_1m_delins_30x_hifi" "default|cfg4_1m_delins_30x_hifi" "lwu2|cfg4_1m_delins_30x_hifi"
