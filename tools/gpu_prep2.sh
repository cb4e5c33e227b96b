#!/bin/bash
# two-wave SHA-512 front end: parity on every latency-path test, then A/B
# against the one-wave front end (front_ms, quad DSM, ring point)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_sha512_gpu.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/pytest_prep2.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/pytest_prep2.log; exit 1; }
tail -3 gpurun_out/pytest_prep2.log
timeout -k 10 600 python3 -u tools/ab_quad.py firedancer_amd/variants/libprep1.so firedancer_amd/libfd_ed25519_gpu.so --rounds 3 --nb 2000 > gpurun_out/ab_prep2.jsonl 2>&1; cat gpurun_out/ab_prep2.jsonl
