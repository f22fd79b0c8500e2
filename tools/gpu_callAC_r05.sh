#!/bin/bash
# Round 5, call AC: engine 0.23.4 -- trace + HBM / SQ PMC passes of the cfg2 and cfg3 steps
# (traffic.json) and the rank slices of the 8-GPU cfg4 split.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/r05_AC
mkdir -p "$OUT"
export TMPDIR=/tmp
for r in 0 3 7; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-cold --emulate-shard 8:$r \
    > "$OUT/shard_$r.log" 2>&1 || { echo "shard $r failed"; tail -5 "$OUT/shard_$r.log"; exit 1; }
  python - "$r" "$OUT/shard_$r.log" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(f"rank {sys.argv[1]} of 8: {d['ms_per_step']:.4f} ms per step")
PY
done
bash tools/gpu_profile.sh r05_AC_cfg2 --inflight 1 --workload cfg2_10kdel_30x_ont || exit $?
bash tools/gpu_profile.sh r05_AC_cfg3 --inflight 1 --workload cfg3_50k_delins_30x_ont || exit $?
echo done
