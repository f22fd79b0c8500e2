#!/bin/bash
# Round 5, call AH: a locus's two windows interleaved (window 2 li + w, SVT_WIN_ILV) -- the whole
# -m gpu suite
# tests, then cfg4 and rank-3 bench lines against variants/v0234.so, alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/r05_AH
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
  tests > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
line() {  # tag log
  python - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
ph = d["roofline"]["phases"]
print(f"{sys.argv[1]:>28}: step {d['ms_per_step']:.4f} ms  index {ph['index_ms']:.4f}  refine {ph['refine_ms']:.4f}")
PY
}
for rep in 1 2; do
  for v in new v0234; do
    lib=""; [ $v != new ] && lib=$PWD/variants/$v.so
    for args in "--inflight 1" "" "--emulate-shard 8:3"; do
      tag="${v}_$(echo "$args" | tr -c 'a-z0-9' '_')_$rep"
      SVTREK_ENGINE_LIB=$lib timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-cold $args \
        > "$OUT/$tag.log" 2>&1 || { echo "$tag failed"; tail -5 "$OUT/$tag.log"; exit 1; }
      line "$tag" "$OUT/$tag.log"
    done
  done
done
echo done
