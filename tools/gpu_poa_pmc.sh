#!/bin/bash
# Run ON THE GPU BOX: SQ counter pass over the POA bench (one rocprofv3 --pmc run).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/poa_pmc_${1:-x}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$OLDPWD}"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU \
  SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS --output-format csv -d "$OUT" -o poa -- \
  python tools/bench_poa.py --repeat 1 --cpu-sample 1 --check 1 > "$OUT/bench.json" 2> "$OUT/err.log"
rc=$?
find "$OUT" -name "*counter_collection*" | head -3
exit $rc
