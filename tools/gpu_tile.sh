#!/bin/bash
# GPU session for the verify-tile work: gpu tests, then the C5 stream bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo TESTS FAILED; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -25 gpurun_out/pytest_gpu.log
timeout -k 10 300 python3 -u tools/bench_tile.py --seconds 10 > gpurun_out/bench_tile.json 2> gpurun_out/bench_tile.err || { echo TILE BENCH FAILED; tail -30 gpurun_out/bench_tile.err; exit 1; }
cat gpurun_out/bench_tile.json
