#!/bin/bash
# Round 4, session E: the eight-lane DSM (fd_k_dsm_oct).  The exchange
# primitive's semantics first, then the field-product and parity tests that
# cover the oct schedule, then the per-signature drop-in's latency.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 ./tools/build/permlane_probe > gpurun_out/permlane.txt 2>&1; rc=$?; cat gpurun_out/permlane.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 python3 -u -m pytest tests/test_fe_gpu.py tests/test_gpu_parity.py tests/test_gpu_host.py tests/test_strict.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_oct.log 2>&1 || { echo OCT TESTS FAILED; grep -E "FAILED|Error|assert" gpurun_out/pytest_oct.log | head -30; tail -40 gpurun_out/pytest_oct.log; exit 1; }
tail -3 gpurun_out/pytest_oct.log
timeout -k 10 300 ./tools/build/per_sig_threads 2000 > gpurun_out/per_sig_oct.jsonl 2> gpurun_out/per_sig_oct.err || { echo PERSIG FAILED; tail -20 gpurun_out/per_sig_oct.err; exit 1; }
cat gpurun_out/per_sig_oct.jsonl
: > gpurun_out/front_tail.jsonl
for n in 1 4096; do
  FD_ED25519_LIB=$PWD/firedancer_amd/variants/lib_fstamps.so timeout -k 10 120 python3 -u tools/front_lone.py 50 $n >> gpurun_out/front_tail.jsonl 2> gpurun_out/front_tail.err || { echo FRONT FAILED; tail -20 gpurun_out/front_tail.err; exit 1; }
done
cat gpurun_out/front_tail.jsonl
