#!/bin/bash
# Run ON THE GPU BOX: the parity / workload GPU tests on the default engine, then one bench line
# per "variant|workload|extra bench args" (variant: variants/NAME.so, or "default").  One time
# limit per step; stops at the first failure.   tools/gpu_ab_pairs.sh TAG SPEC [SPEC ...]
set -u
TAG=${1:?tag}; shift
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -z "${NO_TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_gpu_workloads.py tests/test_gpu_api.py > "$OUT/pytest.log" 2>&1
  rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
fi
for spec in "$@"; do
  v=${spec%%|*}; rest=${spec#*|}; wl=${rest%%|*}; extra=${rest#*|}; [ "$extra" = "$rest" ] && extra=""
  lib=$PWD/svtrek_amd/libsvtrek_hip.so; [ "$v" != default ] && lib=$PWD/variants/$v.so
  n="${v}_${wl}$(echo "$extra" | tr -c 'a-zA-Z0-9' '_')"
  SVTREK_ENGINE_LIB=$lib timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-cold \
    --workload "$wl" $extra > "$OUT/$n.log" 2>&1 || { echo "$n failed rc=$?"; tail -5 "$OUT/$n.log"; exit 1; }
  python - "$n" "$OUT/$n.log" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
ph = d["roofline"]["phases"]
print(f"{sys.argv[1]:>60}: step {d['ms_per_step']:.4f} ms  index {ph['index_ms']:.4f}  refine {ph['refine_ms']:.4f}")
PY
done
