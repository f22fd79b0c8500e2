#!/bin/bash
# Round-4 closing profiles (engine 0.20): trace + PMC passes of the long-read BASELINE workloads,
# the 8-GPU per-rank slices, and an inflate occupancy A/B.  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
bash tools/gpu_profile.sh r04F_cfg5 --workload cfg5_100k_60x_ul_ont && \
bash tools/gpu_profile.sh r04F_cfg3 --workload cfg3_50k_delins_30x_ont && \
bash tools/gpu_profile.sh r04F_cfg2 --workload cfg2_10kdel_30x_ont && \
bash tools/gpu_profile.sh r04F_cfg1 --workload cfg1_100del_10x && \
B='python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-cold' && \
bash tools/gpu_steps.sh r04F_sh "r0|200|$B --emulate-shard 8:0" "r3|200|$B --emulate-shard 8:3" "r7|200|$B --emulate-shard 8:7" \
  'w6|200|SVTREK_ENGINE_LIB=$PWD/variants/inf_w6.so python tools/bench_inflate.py --scale 0.1 --reps 3' \
  'w7|200|SVTREK_ENGINE_LIB=$PWD/variants/inf_w7.so python tools/bench_inflate.py --scale 0.1 --reps 3' \
  'w6b|200|SVTREK_ENGINE_LIB=$PWD/variants/inf_w6.so python tools/bench_inflate.py --scale 0.1 --reps 3' \
  'w7b|200|SVTREK_ENGINE_LIB=$PWD/variants/inf_w7.so python tools/bench_inflate.py --scale 0.1 --reps 3'
