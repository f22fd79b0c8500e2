set -u
mkdir -p gpurun_out/r03t
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_workloads.py > gpurun_out/r03t/pytest.log 2>&1 && tail -2 gpurun_out/r03t/pytest.log && \
VARIANT_WORKLOADS="cfg5_100k_60x_ul_ont cfg3_50k_delins_30x_ont cfg4_1m_delins_30x_hifi" bash tools/gpu_variants.sh r03t_var
