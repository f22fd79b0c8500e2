#!/bin/bash
# Run ON THE GPU BOX (via gpurun): kernel trace + stats and HBM PMC passes of bench.py.
#   tools/gpu_profile.sh TAG [bench args...]
# Writes gpurun_out/prof_TAG/{trace,pmc_fetch,pmc_write,pmc_rdreq,pmc_dram}/ and bench logs.
# Every GPU step has its own time limit and the script stops at the first failing step.
set -u
TAG=${1:?tag}; shift
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS=("$@")
step() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] $name" >> "$OUT/steps.log"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" >> "$OUT/steps.log"
  if [ $rc -ne 0 ]; then echo "step $name failed rc=$rc"; tail -20 "$OUT/$name.log"; exit $rc; fi
}
B=(python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-cold "${ARGS[@]}")
step trace 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
  python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-cold "${ARGS[@]}"
step trace1 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace1" -o run -- \
  python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-cold --inflight 1 "${ARGS[@]}"
step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- "${B[@]}"
step pmc_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- "${B[@]}"
step pmc_rdreq 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum \
  --output-format csv -d "$OUT/pmc_rdreq" -o run -- "${B[@]}"
step pmc_dram 300 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_DRAM_32B_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum \
  --output-format csv -d "$OUT/pmc_dram" -o run -- "${B[@]}"
step pmc_sq 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU \
  SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS --output-format csv -d "$OUT/pmc_sq" -o run -- "${B[@]}"
python tools/trim_prof.py "$OUT"   # (under gpurun's 64 MiB copy-back cap: no per-dispatch traces, engine kernels only)
echo "profile $TAG done"
