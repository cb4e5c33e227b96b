#!/bin/bash
# Round 4, rebuilt final tree: the bench's kernel-trace profile and the
# per-signature thread sweep, beside the v11 bench line.
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu --no-latency > $R/gpurun_out/prof_bench.json 2> $R/gpurun_out/prof.err ) || { echo PROF FAILED; tail -30 gpurun_out/prof.err; exit 1; }
head -8 gpurun_out/prof/run_kernel_stats.csv | cut -c1-200
timeout -k 10 300 ./tools/build/per_sig_threads 2000 > gpurun_out/per_sig_v11.jsonl 2> gpurun_out/per_sig_v11.err || { echo PERSIG FAILED; tail -20 gpurun_out/per_sig_v11.err; exit 1; }
cat gpurun_out/per_sig_v11.jsonl
