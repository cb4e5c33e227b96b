# per-signature drop-in: latency by message size, then the same calls under a
# kernel + memory-copy trace and the per-call device timeline
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python3 -u tools/per_sig_trace.py --calls 300 > gpurun_out/per_sig.json 2> gpurun_out/per_sig.err || { echo PERSIG FAILED; tail -20 gpurun_out/per_sig.err; exit 1; }
cat gpurun_out/per_sig.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pstrace -o run -- python3 $GRAFT_REPO_ROOT/tools/per_sig_trace.py --calls 300 > $GRAFT_REPO_ROOT/gpurun_out/per_sig_traced.json 2> $GRAFT_REPO_ROOT/gpurun_out/pstrace.err || { echo TRACE FAILED; tail -20 $GRAFT_REPO_ROOT/gpurun_out/pstrace.err; exit 1; }
cd $GRAFT_REPO_ROOT
python3 tools/per_sig_trace.py --timeline gpurun_out/pstrace | tee gpurun_out/per_sig_timeline.json
