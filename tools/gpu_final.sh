#!/bin/bash
# Run ON THE GPU BOX: the round's closing measurements -- kernel trace + HBM / SQ PMC passes of
# bench.py on cfg4 and cfg5 (tools/gpu_profile.sh), then the default bench line with the CPU
# baseline, and the per-rank slices of an 8-GPU cfg4 run on this one GPU.  Stops at the first
# failing step.   tools/gpu_final.sh TAG
set -u
TAG=${1:?tag}
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/final_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
bash tools/gpu_profile.sh "${TAG}_cfg4" || exit $?
bash tools/gpu_profile.sh "${TAG}_cfg5" --workload cfg5_100k_60x_ul_ont || exit $?
echo "[$(date +%T)] bench" >> "$OUT/steps.log"
timeout -k 10 400 python3 bench.py > "$OUT/bench.log" 2>&1 || { echo "bench failed"; tail -20 "$OUT/bench.log"; exit 1; }
echo "[$(date +%T)] bench done" >> "$OUT/steps.log"
tail -1 "$OUT/bench.log" | cut -c1-300
for spec in "shard8_r0|--emulate-shard 8:0" "shard8_r7|--emulate-shard 8:7" "scale0125|--scale 0.125"; do
  n=${spec%%|*}; a=${spec#*|}
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-cold $a > "$OUT/cfg4_$n.log" 2>&1 \
    || { echo "$n failed"; tail -5 "$OUT/cfg4_$n.log"; exit 1; }
  echo "[$(date +%T)] cfg4_$n done" >> "$OUT/steps.log"
done
echo "final $TAG done"
