#!/bin/bash
# Run ON THE GPU BOX: SQ/TCC counter passes on bench.py (each pass its own process).
#   tools/gpu_counters.sh TAG "COUNTERS PASS 1" ["COUNTERS PASS 2" ...]
set -u
TAG=${1:?tag}; shift
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/ctr_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > "$OUT/counters_avail.txt" 2>&1 || true
i=0
for pass in "$@"; do
  i=$((i+1))
  echo "[$(date +%T)] pass $i: $pass" >> "$OUT/steps.log"
  timeout -k 10 300 rocprofv3 --pmc $pass --output-format csv -d "$OUT/p$i" -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "[$(date +%T)] pass $i rc=$rc" >> "$OUT/steps.log"
  if [ $rc -ne 0 ]; then tail -20 "$OUT/p$i.log"; exit $rc; fi
done
echo "counters $TAG done"
