#!/bin/bash
# Quad-DSM change check: all GPU tests, 4,096-signature kernel times and
# the ring, HEAD build (variants/lib_old.so) vs the working tree, then C3
# 10M on the quad DSM in both message shapes.
set -o pipefail
mkdir -p gpurun_out
O=firedancer_amd/variants/lib_old.so; N=firedancer_amd/libfd_ed25519_gpu.so
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for r in 1 2 3; do for L in $O $N; do FD_ED25519_LIB=$L timeout -k 10 120 python3 -u tools/time_kernels.py 4096 2> gpurun_out/tk.err || exit 1; done; done
bash tools/ab_ring.sh "--batches 4000 --depths 8 --groups 4 --window-abs 6,7" $O $N || exit 1
timeout -k 10 500 python3 -u tools/c3_adversarial.py --shape txn --schedules ${C3_TXN_SCHED:-quad} > gpurun_out/c3_txn.log 2>&1 || { echo C3 TXN FAILED; tail -5 gpurun_out/c3_txn.log; exit 1; }
tail -1 gpurun_out/c3_txn.log | cut -c1-200
timeout -k 10 500 python3 -u tools/c3_adversarial.py --shape packed --schedules quad > gpurun_out/c3_packed.log 2>&1 || { echo C3 PACKED FAILED; tail -5 gpurun_out/c3_packed.log; exit 1; }
tail -1 gpurun_out/c3_packed.log | cut -c1-200
