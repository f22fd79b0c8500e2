#!/bin/bash
# Run ON THE GPU BOX: two SQ counter passes per engine library (instruction mix and stalls of
# every kernel of the step), bench args as given.   tools/gpu_ixpmc.sh TAG LIB.so [LIB.so ...] [-- bench args]
set -u
TAG=${1:?tag}; shift
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
LIBS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do LIBS+=("$1"); shift; done
[ "${1:-}" = "--" ] && shift
P1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES"
P2="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_WAVES"
for lib in "${LIBS[@]}"; do
  name=$(basename "$lib" .so)
  i=0
  for pass in "$P1" "$P2"; do
    i=$((i+1))
    SVTREK_ENGINE_LIB=$PWD/$lib timeout -s KILL 200 rocprofv3 --pmc $pass --output-format csv -d "$OUT/${name}_p$i" -o run -- \
      python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-cold --no-verify "$@" > "$OUT/${name}_p$i.log" 2>&1 \
      || { echo "fail $name p$i"; tail -5 "$OUT/${name}_p$i.log"; exit 1; }
  done
  echo "done $name"
done
