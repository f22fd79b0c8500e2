#!/bin/bash
# Run ON THE GPU BOX: the index / workload parity tests, then bench every variants/*.so on the
# workloads in AB_WORKLOADS (default cfg4).   tools/gpu_ab.sh TAG
set -u
TAG=${1:?tag}
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out/$TAG
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_workloads.py > gpurun_out/$TAG/pytest.log 2>&1 && tail -2 gpurun_out/$TAG/pytest.log && \
VARIANT_WORKLOADS="${AB_WORKLOADS:-cfg4_1m_delins_30x_hifi}" bash tools/gpu_variants.sh ${TAG}_var
