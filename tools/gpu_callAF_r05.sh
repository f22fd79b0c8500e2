#!/bin/bash
# Round 5, call AF: steps in flight 2 / 3 / 4 (bench.py --inflight K: K engine contexts on K
# streams) on cfg4, rank 3 of 8 and cfg2, alternating, engine 0.23.4.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/r05_AF
mkdir -p "$OUT"
export TMPDIR=/tmp
line() {  # tag log
  python - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
ph = d["roofline"]["phases"]
print(f"{sys.argv[1]:>28}: step {d['ms_per_step']:.4f} ms  index {ph['index_ms']:.4f}  refine {ph['refine_ms']:.4f}  verified {d.get('records_verified')}")
PY
}
for rep in 1 2; do
  for args in "" "--emulate-shard 8:3" "--workload cfg2_10kdel_30x_ont"; do
    for k in 2 3 4; do
      tag="k${k}_$(echo "$args" | tr -c 'a-z0-9' '_')_$rep"
      timeout -k 10 300 python bench.py --steps 30 --warmup 4 --no-cpu-baseline --no-cold --inflight $k $args \
        > "$OUT/$tag.log" 2>&1 || { echo "$tag failed"; tail -5 "$OUT/$tag.log"; exit 1; }
      line "$tag" "$OUT/$tag.log"
    done
  done
done
echo done
