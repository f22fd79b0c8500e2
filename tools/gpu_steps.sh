#!/bin/bash
# Run ON THE GPU BOX (via gpurun): a list of named steps, each under its own time limit;
# stops at the first step that fails, crashes or times out.
#   tools/gpu_steps.sh TAG 'name|seconds|command' ['name|seconds|command' ...]
# Logs: gpurun_out/TAG/<name>.log, gpurun_out/TAG/steps.log.
set -u
TAG=${1:?tag}; shift
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for spec in "$@"; do
  name=${spec%%|*}; rest=${spec#*|}; t=${rest%%|*}; cmd=${rest#*|}
  echo "[$(date +%T)] start $name ($t s): $cmd" | tee -a "$OUT/steps.log"
  timeout -k 10 "$t" bash -c "$cmd" > "$OUT/$name.log" 2>&1
  rc=$?
  echo "[$(date +%T)] end $name rc=$rc" | tee -a "$OUT/steps.log"
  tail -3 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then echo "step $name failed rc=$rc"; exit $rc; fi
done
echo "all steps ok"
