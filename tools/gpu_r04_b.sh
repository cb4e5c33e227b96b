#!/bin/bash
# Round 4, session B: the bench (ring legs with every code checked, the
# open-loop sweep), its kernel-trace profile, the quad-DSM stamps (lone and
# under the ring), and the C5 verify-tile stream in the copy and in-place
# modes.  Each GPU step has its own limit; the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_verify_tile.py tests/test_verify_tile_task.py tests/test_gpu_host.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_tile.log 2>&1 || { echo TILE TESTS FAILED; tail -30 gpurun_out/pytest_tile.log; exit 1; }
tail -3 gpurun_out/pytest_tile.log
timeout -k 10 400 python3 -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH FAILED; tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json | cut -c1-600
R=$GRAFT_REPO_ROOT
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu --no-latency > $R/gpurun_out/prof_bench.json 2> $R/gpurun_out/prof.err ) || { echo PROF FAILED; tail -30 gpurun_out/prof.err; exit 1; }
cat gpurun_out/prof/run_kernel_stats.csv | cut -c1-200
FD_ED25519_LIB=$R/firedancer_amd/variants/lib_qstamps.so timeout -k 10 240 python3 -u tools/quad_stamps.py 3000 > gpurun_out/quad_stamps.jsonl 2> gpurun_out/quad_stamps.err || { echo STAMPS FAILED; tail -20 gpurun_out/quad_stamps.err; exit 1; }
cat gpurun_out/quad_stamps.jsonl
: > gpurun_out/tile_c5.jsonl
for m in "" "--inplace" "--inplace --multi --tiles 2"; do
  for b in 4096 65536 262144; do
    timeout -k 10 120 python3 -u tools/bench_tile.py --sigs 524288 --batch $b --seconds 8 --tiles 1 $m >> gpurun_out/tile_c5.jsonl 2>> gpurun_out/tile_c5.err || { echo TILE FAILED; tail -20 gpurun_out/tile_c5.err; exit 1; }
  done
done
cut -c1-400 gpurun_out/tile_c5.jsonl
