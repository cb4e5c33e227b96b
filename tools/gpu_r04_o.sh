#!/bin/bash
# Round 4, session O: small staged batches (n <= 64) read by the kernels
# from the slot's mapped pinned buffer, no H2D copy: the latency-path,
# portable, strict and teardown GPU tests, then the per-signature A/B
# (FD_ED25519_GPU_IN_DIRECT_MAX=0: the SDMA copy as before), two rounds.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_teardown.py tests/test_gpu_parity.py tests/test_strict.py tests/test_portable.py tests/test_fe_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_o.log 2>&1 || { echo TESTS FAILED; grep -E "FAILED|Error" gpurun_out/pytest_o.log | head -30; tail -40 gpurun_out/pytest_o.log; exit 1; }
tail -3 gpurun_out/pytest_o.log
: > gpurun_out/per_sig_o.jsonl
for r in 1 2; do
  for m in 0 64; do
    FD_ED25519_GPU_IN_DIRECT_MAX=$m timeout -k 10 200 ./tools/build/per_sig_threads 2000 2> gpurun_out/per_sig_o.err | sed "s/^{/{\"in_direct_max\": $m, \"round\": $r, /" >> gpurun_out/per_sig_o.jsonl || { echo PERSIG FAILED; tail -20 gpurun_out/per_sig_o.err; exit 1; }
  done
done
cut -c1-220 gpurun_out/per_sig_o.jsonl
