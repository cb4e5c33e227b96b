#!/bin/bash
# Round 4, session P: every stream a batch can take is warmed at engine
# creation (fd_stream_warm); the engine-host, parity and teardown GPU
# tests, then the per-signature runs twice (with copies of every size class; the 16-thread maximum was
# 8.7-9.1 ms: a third group-commit leader's first use of its slot).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_teardown.py tests/test_gpu_parity.py tests/test_gpu_host.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_p.log 2>&1 || { echo TESTS FAILED; grep -E "FAILED|Error" gpurun_out/pytest_p.log | head -30; tail -40 gpurun_out/pytest_p.log; exit 1; }
tail -3 gpurun_out/pytest_p.log
: > gpurun_out/per_sig_p.jsonl
for r in 1 2; do
  timeout -k 10 200 ./tools/build/per_sig_threads 2000 2> gpurun_out/per_sig_p.err | sed "s/^{/{\"round\": $r, /" >> gpurun_out/per_sig_p.jsonl || { echo PERSIG FAILED; tail -20 gpurun_out/per_sig_p.err; exit 1; }
done
cut -c1-200 gpurun_out/per_sig_p.jsonl
