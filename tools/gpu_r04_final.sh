#!/bin/bash
# Round 4, final tree: the whole GPU suite, smoke and the bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_final.log 2>&1 || { echo GPU TESTS FAILED; grep -E "FAILED|Error" gpurun_out/pytest_final.log | head -30; tail -40 gpurun_out/pytest_final.log; exit 1; }
tail -3 gpurun_out/pytest_final.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1 || { echo SMOKE FAILED; tail -20 gpurun_out/smoke_final.log; exit 1; }
tail -1 gpurun_out/smoke_final.log
timeout -k 10 400 python3 -u bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || { echo BENCH FAILED; tail -30 gpurun_out/bench_final.err; exit 1; }
cut -c1-400 gpurun_out/bench_final.json
