#!/bin/bash
# Round 4, session G: the eight-lane DSM with its prologue on half field
# elements -- oct parity again, the per-signature latency, the latency
# DSMs' clock, and the front end's tail stamps (sc_reduce vs recoder).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_fe_gpu.py tests/test_gpu_parity.py tests/test_strict.py tests/test_gpu_host.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_oct3.log 2>&1 || { echo OCT TESTS FAILED; grep -E "FAILED|Error|assert" gpurun_out/pytest_oct3.log | head -30; tail -40 gpurun_out/pytest_oct3.log; exit 1; }
tail -3 gpurun_out/pytest_oct3.log
timeout -k 10 300 ./tools/build/per_sig_threads 2000 > gpurun_out/per_sig_oct3.jsonl 2> gpurun_out/per_sig_oct3.err || { echo PERSIG FAILED; tail -20 gpurun_out/per_sig_oct3.err; exit 1; }
cat gpurun_out/per_sig_oct3.jsonl
timeout -k 10 120 python3 -u tools/oct_clock.py 300 > gpurun_out/oct_clock3.json 2> gpurun_out/oct_clock3.err || { echo CLOCK FAILED; tail -20 gpurun_out/oct_clock3.err; exit 1; }
cat gpurun_out/oct_clock3.json
: > gpurun_out/front_tail2.jsonl
for n in 1 4096; do
  FD_ED25519_LIB=$PWD/firedancer_amd/variants/lib_fstamps.so timeout -k 10 120 python3 -u tools/front_lone.py 50 $n >> gpurun_out/front_tail2.jsonl 2> gpurun_out/front_tail2.err || { echo FRONT FAILED; tail -20 gpurun_out/front_tail2.err; exit 1; }
done
cut -c1-1500 gpurun_out/front_tail2.jsonl
