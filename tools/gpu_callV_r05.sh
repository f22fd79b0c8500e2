#!/bin/bash
# Round 5, call V: kernel trace + HBM / SQ PMC passes of engine 0.23.2 (the benched build) on
# cfg4 and cfg2, one step in flight (kernel durations without the other context's overlap), for
# profiles/traffic.json (tools/make_traffic.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
bash tools/gpu_profile.sh r05_V_cfg4 --inflight 1 || exit $?
bash tools/gpu_profile.sh r05_V_cfg2 --inflight 1 --workload cfg2_10kdel_30x_ont || exit $?
echo done
