#!/bin/bash
# One GPU session: tests, smoke, bench, kernel-trace profile.  Each GPU step
# has its own time limit; the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
STAGE=${1:-all}
if [[ $STAGE == all || $STAGE == test ]]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
  tail -20 gpurun_out/pytest_gpu.log
  timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE FAILED; cat gpurun_out/smoke.log; exit 1; }
  cat gpurun_out/smoke.log
fi
if [[ $STAGE == all || $STAGE == bench ]]; then
  timeout -k 10 300 python3 -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH FAILED; tail -30 gpurun_out/bench.err; exit 1; }
  cat gpurun_out/bench.json
fi
if [[ $STAGE == all || $STAGE == prof ]]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 2 --no-cpu --no-latency > $GRAFT_REPO_ROOT/gpurun_out/prof_bench.json 2> $GRAFT_REPO_ROOT/gpurun_out/prof.err || { echo PROF FAILED; tail -30 $GRAFT_REPO_ROOT/gpurun_out/prof.err; exit 1; }
  cd $GRAFT_REPO_ROOT
  find gpurun_out/prof -name "*stats*" | head; cat $(find gpurun_out/prof -name "*kernel_stats.csv" | head -1) | cut -c1-250
fi
