#!/bin/bash
# Round 4, session D: the DSM clock accumulators (GPU test), then the bench
# with the effective clock in its roofline, and its kernel-trace profile.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_host.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_host.log 2>&1 || { echo HOST TESTS FAILED; tail -30 gpurun_out/pytest_host.log; exit 1; }
tail -3 gpurun_out/pytest_host.log
timeout -k 10 400 python3 -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH FAILED; tail -30 gpurun_out/bench.err; exit 1; }
cut -c1-300 gpurun_out/bench.json
R=$GRAFT_REPO_ROOT
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu --no-latency > $R/gpurun_out/prof_bench.json 2> $R/gpurun_out/prof.err ) || { echo PROF FAILED; tail -30 gpurun_out/prof.err; exit 1; }
head -4 gpurun_out/prof/run_kernel_stats.csv | cut -c1-200
