#!/bin/bash
# Round 5, call AB: engine 0.23.4 on a fresh box -- the whole -m gpu suite, smoke(), the default
# bench line, then the trace + HBM / SQ PMC passes of the cfg4 step (traffic.json).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/r05_AB
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 560 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests \
  > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -5 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 300 python bench.py > "$OUT/bench.log" 2>&1 || { tail -5 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log" | cut -c1-300
bash tools/gpu_profile.sh r05_AB_cfg4 --inflight 1 || exit $?
echo done
