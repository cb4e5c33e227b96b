#!/bin/bash
# Round 4, session K: the oct DSM's operand exchange, A/B by main-loop
# cycles per single-signature wave: 0 = permlane copy/swap/select for g,
# 1 = g partner limbs by ds_swizzle (the product), 2 = partner limbs sent
# pre-scaled (19 g or g) so the swizzle results feed the MACs; two rounds.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/oct_ab.jsonl
for r in 1 2; do for v in 0 1 2; do
  FD_ED25519_LIB=$PWD/firedancer_amd/variants/lib_oct$v.so timeout -k 10 120 python3 -u tools/oct_clock.py 400 > gpurun_out/oct_ab_one.json 2> gpurun_out/oct_ab.err || { echo FAILED $v; tail -20 gpurun_out/oct_ab.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/oct_ab_one.json')); d['variant']=$v; print(json.dumps(d))" | tee -a gpurun_out/oct_ab.jsonl
done; done
FD_ED25519_LIB=$PWD/firedancer_amd/variants/lib_oct2.so timeout -k 10 300 python3 -u -m pytest tests/test_fe_gpu.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "fe or oct" > gpurun_out/pytest_oct2v.log 2>&1 || { echo V2 TESTS FAILED; tail -30 gpurun_out/pytest_oct2v.log; exit 1; }
tail -2 gpurun_out/pytest_oct2v.log
