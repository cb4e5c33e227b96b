#!/bin/bash
# lone 4096-signature launches: per-wave front-end stamps (two-wave vs
# one-wave SHA-512 prep), parity of the product build's latency path
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_sha512_gpu.py -m gpu -x -q --timeout 150 --timeout-method thread -k "quad or golden or vectors or sha" > gpurun_out/pytest_front.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/pytest_front.log; exit 1; }
tail -2 gpurun_out/pytest_front.log
for L in firedancer_amd/variants/libst1.so firedancer_amd/variants/libst2.so firedancer_amd/variants/libst1.so firedancer_amd/variants/libst2.so; do
  FD_ED25519_LIB=$PWD/$L timeout -k 10 120 python3 -u tools/front_lone.py 50 >> gpurun_out/front_lone.jsonl 2> gpurun_out/front_lone.err || { echo FAILED $L; tail -20 gpurun_out/front_lone.err; exit 1; }
done
cat gpurun_out/front_lone.jsonl
