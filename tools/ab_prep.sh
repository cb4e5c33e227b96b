# prep/front-end check: parity tests + serial kernel times (262,144: fd_k_prep; 4,096: fd_k_front) vs a previous build
set -o pipefail
mkdir -p gpurun_out
O=firedancer_amd/variants/lib_old.so; N=firedancer_amd/libfd_ed25519_gpu.so
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pp_pytest.log 2>&1 || { echo PYTEST FAILED; tail -30 gpurun_out/pp_pytest.log; exit 1; }
tail -1 gpurun_out/pp_pytest.log
for r in 1 2 3; do for L in $O $N; do
  FD_ED25519_LIB=$L timeout -k 10 120 python3 -u tools/time_kernels.py 262144 2> gpurun_out/tk.err || exit 1
  FD_ED25519_LIB=$L timeout -k 10 120 python3 -u tools/time_kernels.py 4096 2> gpurun_out/tk.err || exit 1
done; done
