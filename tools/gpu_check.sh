#!/bin/bash
# Run ON THE GPU BOX: smoke, GPU parity tests, then bench.
# Stops at the first step that crashes / times out; a plain test failure (rc 1) still
# lets the benches run so one call yields both signals.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
TAG=${1:-check}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
run() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] start $name" >> "$OUT/steps.log"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] end $name rc=$rc" >> "$OUT/steps.log"
  return $rc
}
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
run pytest 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread; rc=$?
tail -5 "$OUT/pytest.log"
if [ $rc -gt 1 ]; then echo "pytest crashed rc=$rc"; exit $rc; fi
run bench 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline || exit $?
tail -1 "$OUT/bench.log"
exit $rc
