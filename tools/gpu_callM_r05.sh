#!/bin/bash
# Round 5, call M: where the BGZF inflate kernel's time goes -- the per-block counts and times of
# a -DSVT_PHASE_PROF=1 build (variants/x_iprof.so) on cfg2 x 0.1, and SQ counters of one launch.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/r05_M
mkdir -p "$OUT"
export TMPDIR=/tmp
SVTREK_ENGINE_LIB=$PWD/variants/x_iprof.so timeout -k 10 300 python tools/bench_inflate.py --scale 0.1 --reps 2 --phase \
  > "$OUT/inf_prof.log" 2>&1 || { echo "prof failed"; tail -5 "$OUT/inf_prof.log"; exit 1; }
tail -1 "$OUT/inf_prof.log"
P1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_WAIT_ANY"
timeout -s KILL 200 rocprofv3 --pmc $P1 --output-format csv -d "$OUT/pmc1" -o run -- \
  python3 tools/bench_inflate.py --scale 0.1 --reps 1 > "$OUT/pmc1.log" 2>&1 || { echo "pmc failed"; exit 1; }
P2="SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_SALU SQ_WAVES SQ_BUSY_CYCLES"
timeout -s KILL 200 rocprofv3 --pmc $P2 --output-format csv -d "$OUT/pmc2" -o run -- \
  python3 tools/bench_inflate.py --scale 0.1 --reps 1 > "$OUT/pmc2.log" 2>&1 || { echo "pmc2 failed"; tail -3 "$OUT/pmc2.log"; exit 1; }
echo done
