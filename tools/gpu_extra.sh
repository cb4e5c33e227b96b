#!/bin/bash
# GPU tests, then the non-C2 configs (C1, C4), then the C3 10M run.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo TESTS FAILED; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -5 gpurun_out/pytest_gpu.log
timeout -k 10 400 python3 -u tools/bench_configs.py > gpurun_out/configs.jsonl 2> gpurun_out/configs.err || { echo CONFIGS FAILED; tail -30 gpurun_out/configs.err; exit 1; }
cut -c1-600 gpurun_out/configs.jsonl
if [[ "$1" == c3 ]]; then
  timeout -k 10 600 python3 -u tools/c3_adversarial.py > gpurun_out/c3.log 2>&1 || { echo C3 FAILED; tail -5 gpurun_out/c3.log; exit 1; }
  tail -1 gpurun_out/c3.log | cut -c1-400
fi
