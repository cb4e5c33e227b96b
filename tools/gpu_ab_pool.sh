#!/bin/bash
# Parity tests, then an interleaved throughput A/B (tools/ab.sh) and the
# small-batch kernel times of the HEAD build (variants/lib_old.so) against
# the working tree's library.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
bash tools/ab.sh firedancer_amd/variants/lib_old.so firedancer_amd/libfd_ed25519_gpu.so ${ROUNDS:-3} || exit 1
for r in 1 2; do for L in firedancer_amd/variants/lib_old.so firedancer_amd/libfd_ed25519_gpu.so; do FD_ED25519_LIB=$L timeout -k 10 120 python3 -u tools/time_kernels.py 4096 2> gpurun_out/tk.err || exit 1; done; done
