set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python3 -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH FAILED; tail -30 gpurun_out/bench.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/ring_w8 -o ring -- python3 $GRAFT_REPO_ROOT/tools/ring_trace.py --window 8 > $GRAFT_REPO_ROOT/gpurun_out/ring_w8.json 2> $GRAFT_REPO_ROOT/gpurun_out/ring_w8.err || { echo TRACE FAILED; exit 1; }
cat $GRAFT_REPO_ROOT/gpurun_out/ring_w8.json
