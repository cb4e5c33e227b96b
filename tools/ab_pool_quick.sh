# pool-path check: pooled-DSM parity tests + throughput A/B against a previous build
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pq_pytest.log 2>&1 || { echo PYTEST FAILED; tail -30 gpurun_out/pq_pytest.log; exit 1; }
tail -1 gpurun_out/pq_pytest.log
bash tools/ab.sh firedancer_amd/variants/lib_old.so firedancer_amd/libfd_ed25519_gpu.so 3
