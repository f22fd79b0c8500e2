#!/bin/bash
# Run ON THE GPU BOX: per-variant instruction counters of the timed kernel (one --pmc pass
# per library: the default engine and every svtrek_amd/diag/*.so), bench args as given.
#   tools/gpu_pmc_diag.sh TAG [bench args...]
set -u
TAG=${1:?tag}; shift
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/pmcdiag_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for lib in svtrek_amd/libsvtrek_hip.so svtrek_amd/diag/*.so; do
  name=$(basename "$lib" .so)
  SVTREK_ENGINE_LIB=$PWD/$lib timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
    --output-format csv -d "$OUT/$name" -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-cold --no-verify "$@" > "$OUT/$name.log" 2>&1 || { echo "fail $name"; tail -5 "$OUT/$name.log"; exit 1; }
  echo "done $name"
done
