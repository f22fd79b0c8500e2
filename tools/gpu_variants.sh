#!/bin/bash
# Run ON THE GPU BOX: bench each variants/*.so (one time limit per run, stop at the first crash)
# and print the index / refine phase times.   tools/gpu_variants.sh TAG [bench args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
TAG=${1:?tag}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
WL=${VARIANT_WORKLOADS:-cfg4_1m_delins_30x_hifi}
for wl in $WL; do
for so in variants/*.so; do
  n=$(basename "$so" .so)_$wl
  SVTREK_ENGINE_LIB=$PWD/$so timeout -k 10 240 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-cold --workload $wl "$@" \
    > "$OUT/$n.log" 2>&1 || { echo "$n failed rc=$?"; tail -5 "$OUT/$n.log"; exit 1; }
  python - "$n" "$OUT/$n.log" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
ph = d["roofline"]["phases"]
print(f"{sys.argv[1]:>40}: step {d['ms_per_step']:.4f} ms  index {ph['index_ms']:.4f}  refine {ph['refine_ms']:.4f}  verified {d.get('records_verified')}")
PY
done
done
