set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/quad_scale_probe.py || exit 1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_c3_10m.py tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 500 --timeout-method thread > gpurun_out/direct_pytest.log 2>&1 || { echo PYTEST FAILED; tail -30 gpurun_out/direct_pytest.log; exit 1; }
tail -2 gpurun_out/direct_pytest.log
