#!/bin/bash
# Round 4, session Q: small staged batches copied in by a kernel on their
# own stream (fd_k_stage) instead of SDMA; slot buffers now mapped and
# coherent.  GPU tests of the paths that stage, the per-signature A/B
# (FD_ED25519_GPU_STAGE_KERNEL_MAX=0: SDMA as before), two rounds, then the
# bench without the CPU leg (ring legs: SDMA from the coherent buffers).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_teardown.py tests/test_gpu_parity.py tests/test_gpu_host.py tests/test_verify_tile.py tests/test_portable.py tests/test_strict.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_q.log 2>&1 || { echo TESTS FAILED; grep -E "FAILED|Error" gpurun_out/pytest_q.log | head -30; tail -40 gpurun_out/pytest_q.log; exit 1; }
tail -3 gpurun_out/pytest_q.log
: > gpurun_out/per_sig_q.jsonl
for r in 1 2; do
  for m in 0 64; do
    FD_ED25519_GPU_STAGE_KERNEL_MAX=$m timeout -k 10 200 ./tools/build/per_sig_threads 2000 2> gpurun_out/per_sig_q.err | sed "s/^{/{\"stage_kernel_max\": $m, \"round\": $r, /" >> gpurun_out/per_sig_q.jsonl || { echo PERSIG FAILED; tail -20 gpurun_out/per_sig_q.err; exit 1; }
  done
done
cut -c1-200 gpurun_out/per_sig_q.jsonl
timeout -k 10 400 python3 -u bench.py --no-cpu > gpurun_out/bench_q.json 2> gpurun_out/bench_q.err || { echo BENCH FAILED; tail -30 gpurun_out/bench_q.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/bench_q.json')); l=d['latency']
print('value', d['value'], 'frac', d['roofline']['frac'])
print('closed', l['pcie_inclusive_verifies_per_s'], l['p99_ms'], 'w8', l['window8_point']['pcie_inclusive_verifies_per_s'], l['window8_point']['p99_ms'])
print('paced', [(round(p['offered_verifies_per_s']/1e6), round(p['sched_to_done_p99_ms'],3)) for p in l['paced']])
print('depth1', l['depth1']['p50_ms'], l['depth1']['p99_ms'])
"
