#!/bin/bash
# Round 4, session V9: the final tree (batched prologue loads) -- the whole GPU suite, smoke, the
# bench and its kernel-trace profile, and the per-signature device timeline.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo GPU TESTS FAILED; grep -E "FAILED|Error" gpurun_out/pytest_gpu.log | head -30; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python3 -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH FAILED; tail -30 gpurun_out/bench.err; exit 1; }
cut -c1-300 gpurun_out/bench.json
R=$GRAFT_REPO_ROOT
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu --no-latency > $R/gpurun_out/prof_bench.json 2> $R/gpurun_out/prof.err ) || { echo PROF FAILED; tail -30 gpurun_out/prof.err; exit 1; }
head -4 gpurun_out/prof/run_kernel_stats.csv | cut -c1-200
timeout -k 10 300 ./tools/build/per_sig_threads 2000 > gpurun_out/per_sig_v9.jsonl 2> gpurun_out/per_sig_v9.err || { echo PERSIG FAILED; tail -20 gpurun_out/per_sig_v9.err; exit 1; }
cat gpurun_out/per_sig_v9.jsonl
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/pstrace -o run -- python3 $R/tools/per_sig_trace.py --calls 300 > $R/gpurun_out/per_sig_traced.json 2> $R/gpurun_out/pstrace.err ) || { echo TRACE FAILED; tail -20 gpurun_out/pstrace.err; exit 1; }
python3 tools/per_sig_trace.py --timeline gpurun_out/pstrace > gpurun_out/per_sig_timeline.json
cat gpurun_out/per_sig_timeline.json
