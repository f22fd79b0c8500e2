#!/bin/bash
# Round-4 closing run on engine 0.21: smoke, every GPU test, the default bench line, its kernel
# trace, then the cfg4 trace + PMC passes (traffic.json).  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
bash tools/gpu_full.sh r04_I --no-cfg5 && \
bash tools/gpu_profile.sh r04I_cfg4 --workload cfg4_1m_delins_30x_hifi
