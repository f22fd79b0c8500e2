#!/bin/bash
# Run ON THE GPU BOX: lane-kernel width A/B (span1 = one wave per window, W=8, W=32) per workload.
set -u
TAG=${1:?tag}
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/lanew_$TAG
mkdir -p "$OUT"
for wl in cfg2_10kdel_30x_ont cfg3_50k_delins_30x_ont cfg4_1m_delins_30x_hifi; do
  for v in "SVTREK_GATHER=span1" "SVTREK_LANE_W=8" "SVTREK_LANE_W=32"; do
    env $v timeout -k 10 300 python bench.py --workload $wl --steps 20 --warmup 3 --no-cpu-baseline --no-cold > "$OUT/$wl.$v.log" 2>&1 || { echo "fail $wl $v"; tail -5 "$OUT/$wl.$v.log"; exit 1; }
    echo "$wl $v $(python3 -c "import json;d=json.loads(open('$OUT/$wl.$v.log').read().strip().splitlines()[-1]);r=d['roofline'];print(round(d['value']/1e6,1),r['kernel_ms_mean'])")" | tee -a "$OUT/summary.txt"
  done
done
