#!/bin/bash
# Round 5, call J: kernel trace + PMC passes (HBM bytes, SQ issue / wait counters) of the cfg4
# step on the current engine at one step in flight (clean per-kernel durations), then the
# stream walk's range count (SVTREK_IX_RANGES) on cfg2 / cfg3.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/r05_J
mkdir -p "$OUT"
export TMPDIR=/tmp
bash tools/gpu_profile.sh r05_J_cfg4 --workload cfg4_1m_delins_30x_hifi --inflight 1 || exit $?
for wl in cfg2_10kdel_30x_ont cfg3_50k_delins_30x_ont; do
  for nr in 131072 65536 32768 262144; do
    SVTREK_IX_RANGES=$nr timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-cold \
      --workload $wl --inflight 1 > "$OUT/${wl}_r$nr.log" 2>&1 || { echo "$wl $nr failed"; tail -5 "$OUT/${wl}_r$nr.log"; exit 1; }
    python - "$wl r$nr" "$OUT/${wl}_r$nr.log" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
ph = d["roofline"]["phases"]
print(f"{sys.argv[1]:>40}: step {d['ms_per_step']:.4f} ms  index {ph['index_ms']:.4f}  refine {ph['refine_ms']:.4f}")
PY
  done
done
