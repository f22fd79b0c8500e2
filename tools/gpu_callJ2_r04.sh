#!/bin/bash
# Round-4 closing run on engine 0.21.1 (short form): smoke, every GPU test, the default bench
# line and its kernel trace, then the cfg4 trace + PMC passes.  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
bash tools/gpu_full.sh r04_J --no-cfg5 && \
bash tools/gpu_profile.sh r04J_cfg4 --workload cfg4_1m_delins_30x_hifi
