# quad-path front end without the op-stream memset: parity + small-batch times + ring, vs a previous build
set -o pipefail
mkdir -p gpurun_out
O=firedancer_amd/variants/lib_old.so; N=firedancer_amd/libfd_ed25519_gpu.so
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_verify_tile.py -x -q --timeout 200 --timeout-method thread > gpurun_out/fm_pytest.log 2>&1 || { echo PYTEST FAILED; tail -30 gpurun_out/fm_pytest.log; exit 1; }
tail -1 gpurun_out/fm_pytest.log
for r in 1 2; do for L in $O $N; do FD_ED25519_LIB=$L timeout -k 10 120 python3 -u tools/time_kernels.py 4096 2> gpurun_out/tk.err || exit 1; done; done
bash tools/ab_ring.sh "--batches 6000 --depths 8 --groups 4 --window-abs 1,6,7" $O $N || exit 1
