#!/bin/bash
# Timeline of depth-1 4096-signature batches: kernel + memory-copy trace
# (no counters) of tools/latency_breakdown.py, for the per-batch gap analysis.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/lat -o lat -- python3 $GRAFT_REPO_ROOT/${LAT_SCRIPT:-tools/latency_breakdown.py} ${LAT_ARGS:-4096} > $GRAFT_REPO_ROOT/gpurun_out/lat.json 2> $GRAFT_REPO_ROOT/gpurun_out/lat.err || { echo FAILED; tail -20 $GRAFT_REPO_ROOT/gpurun_out/lat.err; exit 1; }
cat $GRAFT_REPO_ROOT/gpurun_out/lat.json
