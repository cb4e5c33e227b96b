#!/bin/bash
# Round 4, session L: the oct product's carry chain after the MACs (0) or
# absorbed into the column sums (1), A/B by main-loop cycles per
# single-signature wave, two rounds; then the oct tests on variant 1.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/oct_chain_ab.jsonl
for r in 1 2; do for v in 0 1; do
  FD_ED25519_LIB=$PWD/firedancer_amd/variants/lib_ch$v.so timeout -k 10 120 python3 -u tools/oct_clock.py 400 > gpurun_out/oct_ab_one.json 2> gpurun_out/oct_ab.err || { echo FAILED $v; tail -20 gpurun_out/oct_ab.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/oct_ab_one.json')); d['chain_variant']=$v; print(json.dumps(d))" | tee -a gpurun_out/oct_chain_ab.jsonl
done; done
FD_ED25519_LIB=$PWD/firedancer_amd/variants/lib_ch1.so timeout -k 10 300 python3 -u -m pytest tests/test_fe_gpu.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "fe or oct" > gpurun_out/pytest_ch1.log 2>&1 || { echo CH1 TESTS FAILED; tail -30 gpurun_out/pytest_ch1.log; exit 1; }
tail -2 gpurun_out/pytest_ch1.log
