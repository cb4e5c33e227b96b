# the C2 ring under a kernel + memory-copy trace (no counters), 6 and 8 in flight
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for W in 6 8; do
  timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/ring_w$W -o ring -- python3 $GRAFT_REPO_ROOT/tools/ring_trace.py --window $W > $GRAFT_REPO_ROOT/gpurun_out/ring_w$W.json 2> $GRAFT_REPO_ROOT/gpurun_out/ring_w$W.err || { echo FAILED; tail -20 $GRAFT_REPO_ROOT/gpurun_out/ring_w$W.err; exit 1; }
  cat $GRAFT_REPO_ROOT/gpurun_out/ring_w$W.json
  python3 $GRAFT_REPO_ROOT/tools/ring_trace.py --analyze $GRAFT_REPO_ROOT/gpurun_out/ring_w$W > $GRAFT_REPO_ROOT/gpurun_out/ring_w$W.analysis.json || exit 1
  cat $GRAFT_REPO_ROOT/gpurun_out/ring_w$W.analysis.json
done
