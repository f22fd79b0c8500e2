#!/bin/bash
# Round 5, call AN: the lane emit with 4 or 2 stream loads per lane per step (SVT_IX2_UE; 8 in-tree)
# -- parity on ue4, cfg4 / rank-3 bench lines alternating, index-only RDREQ passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/r05_AN
mkdir -p "$OUT"
export TMPDIR=/tmp
SVTREK_ENGINE_LIB=$PWD/variants/ue4.so timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_workloads.py > "$OUT/pytest_ue4.log" 2>&1
rc=$?; tail -2 "$OUT/pytest_ue4.log"; [ $rc -eq 0 ] || exit $rc
line() {  # tag log
  python - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
ph = d["roofline"]["phases"]
print(f"{sys.argv[1]:>28}: step {d['ms_per_step']:.4f} ms  index {ph['index_ms']:.4f}  refine {ph['refine_ms']:.4f}")
PY
}
for rep in 1 2; do
  for v in tree ue4 ue2; do
    lib=""; [ $v != tree ] && lib=$PWD/variants/$v.so
    for args in "" "--emulate-shard 8:3"; do
      tag="${v}_$(echo "$args" | tr -c 'a-z0-9' '_')_$rep"
      SVTREK_ENGINE_LIB=$lib timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-cold $args \
        > "$OUT/$tag.log" 2>&1 || { echo "$tag failed"; tail -5 "$OUT/$tag.log"; exit 1; }
      line "$tag" "$OUT/$tag.log"
    done
  done
done
for v in tree ue4 ue2; do
  lib=""; [ $v != tree ] && lib=$PWD/variants/$v.so
  SVTREK_ENGINE_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${v}_trace" -o run -- \
    python3 tools/ix_only.py > "$OUT/${v}_trace.log" 2>&1 || { echo "$v trace failed"; exit 1; }
  SVTREK_ENGINE_LIB=$lib timeout -s KILL 200 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum \
    --output-format csv -d "$OUT/${v}_rdreq" -o run -- python3 tools/ix_only.py > "$OUT/${v}_rdreq.log" 2>&1 || { echo "$v rdreq failed"; exit 1; }
done
echo done
