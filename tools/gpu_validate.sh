#!/bin/bash
# Run ON THE GPU BOX (via gpurun): the round's validation of the committed tree -- the whole -m gpu
# suite, smoke(), the default bench line (with its CPU baseline), rank 3 of an emulated 8-GPU run,
# and a kernel trace of the default bench.   tools/gpu_validate.sh TAG [extra 'name|seconds|cmd' ...]
# (The round-4/5 one-off tools/gpu_call*_r0{4,5}.sh scripts were this sequence with small edits;
# they are in git history.)  Each step runs under its own time limit; the first failure ends it.
set -u
TAG=${1:?tag}; shift
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/$TAG
exec_steps() { bash tools/gpu_steps.sh "$TAG" "$@"; }
exec_steps \
  "pytest|700|python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests" \
  "smoke|120|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench|300|python bench.py" \
  "bench_rank3|300|python bench.py --emulate-shard 8:3 --no-cpu-baseline" \
  "trace|400|rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-cold" \
  "$@"
