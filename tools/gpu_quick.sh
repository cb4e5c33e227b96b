#!/bin/bash
# GPU tests + smoke + a short bench (no CPU/latency legs).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo TESTS FAILED; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -8 gpurun_out/pytest_gpu.log
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE FAILED; cat gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
timeout -k 10 300 python3 -u bench.py --no-cpu --no-latency > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH FAILED; tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
