# Experiment record (profiles/r02_quad_ops_sigmajor.txt): A/B of step-major vs signature-major op
# streams for every DSM, with the since-removed FD_OPS_SIGMAJOR build switch (lib_tmajor.so =
# -DFD_OPS_SIGMAJOR=0).  Kept for the record; the product now uses signature-major streams
# for the quad DSM only.
set -o pipefail
mkdir -p gpurun_out
N=firedancer_amd/libfd_ed25519_gpu.so; O=firedancer_amd/variants/lib_tmajor.so
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ops_pytest.log 2>&1 || { echo PYTEST FAILED; tail -30 gpurun_out/ops_pytest.log; exit 1; }
tail -1 gpurun_out/ops_pytest.log
bash tools/ab.sh $O $N 3 || exit 1
for r in 1 2; do for L in $O $N; do FD_ED25519_LIB=$L timeout -k 10 120 python3 -u tools/time_kernels.py 4096 2> gpurun_out/tk.err || exit 1; FD_ED25519_LIB=$L timeout -k 10 120 python3 -u tools/time_kernels.py 65536 2> gpurun_out/tk.err || exit 1; done; done
bash tools/pmc_lib.sh $O tmajor_fetch FETCH_SIZE || exit 1
bash tools/pmc_lib.sh $N sigmajor_fetch FETCH_SIZE || exit 1
bash tools/pmc_lib.sh $O tmajor_write WRITE_SIZE || exit 1
bash tools/pmc_lib.sh $N sigmajor_write WRITE_SIZE || exit 1
