#!/bin/bash
# Round 5, call AM: the final committed tree again (after the DIAG 23 line; engine 0.23.4, three steps in flight by
# default) on a fresh box -- the whole -m gpu suite, smoke(), the default bench line (with its CPU
# baseline) and a kernel trace of the default bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/r05_AM
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests \
  > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -5 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 300 python bench.py > "$OUT/bench.log" 2>&1 || { tail -5 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log" | cut -c1-300
timeout -k 10 300 python bench.py --emulate-shard 8:3 --no-cpu-baseline > "$OUT/bench_rank3.log" 2>&1 || { tail -5 "$OUT/bench_rank3.log"; exit 1; }
tail -1 "$OUT/bench_rank3.log" | cut -c1-200
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
  python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-cold > "$OUT/bench_trace.log" 2>&1 || { tail -5 "$OUT/bench_trace.log"; exit 1; }
echo done
