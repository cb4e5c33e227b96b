#!/bin/bash
# Round 4, session I: the two-pass recoder in the latency front end --
# parity of everything on the latency path, the front end's tail stamps,
# the per-signature latency and the bench (ring legs).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_sha512_gpu.py tests/test_strict.py tests/test_gpu_configs.py tests/test_gpu_host.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_rec2.log 2>&1 || { echo TESTS FAILED; grep -E "FAILED|Error" gpurun_out/pytest_rec2.log | head -30; tail -40 gpurun_out/pytest_rec2.log; exit 1; }
tail -3 gpurun_out/pytest_rec2.log
: > gpurun_out/front_tail3.jsonl
for n in 1 4096; do
  FD_ED25519_LIB=$PWD/firedancer_amd/variants/lib_fstamps.so timeout -k 10 120 python3 -u tools/front_lone.py 50 $n >> gpurun_out/front_tail3.jsonl 2> gpurun_out/front_tail3.err || { echo FRONT FAILED; tail -20 gpurun_out/front_tail3.err; exit 1; }
done
cut -c1-1200 gpurun_out/front_tail3.jsonl
timeout -k 10 300 ./tools/build/per_sig_threads 2000 > gpurun_out/per_sig_i.jsonl 2> gpurun_out/per_sig_i.err || { echo PERSIG FAILED; tail -20 gpurun_out/per_sig_i.err; exit 1; }
cat gpurun_out/per_sig_i.jsonl
timeout -k 10 400 python3 -u bench.py > gpurun_out/bench_i.json 2> gpurun_out/bench_i.err || { echo BENCH FAILED; tail -30 gpurun_out/bench_i.err; exit 1; }
cut -c1-300 gpurun_out/bench_i.json
