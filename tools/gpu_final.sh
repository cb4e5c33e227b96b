#!/bin/bash
# Final-tree evidence in one call: tests, smoke, bench, kernel-trace profile
# (tools/gpu_round.sh), the C1/C4 configs, and C3 10M on the quad DSM in
# both message shapes.  Every GPU step has its own time limit; the chain
# stops at the first failure.
set -o pipefail
bash tools/gpu_round.sh all > gpurun_out/round.txt 2>&1 || { echo ROUND FAILED; tail -40 gpurun_out/round.txt; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 400 python3 -u tools/bench_configs.py > gpurun_out/configs.jsonl 2> gpurun_out/configs.err || { echo CONFIGS FAILED; tail -30 gpurun_out/configs.err; exit 1; }
timeout -k 10 500 python3 -u tools/c3_adversarial.py --shape txn --schedules ${C3_SCHED:-pool,uniform,quad} > gpurun_out/c3_txn.log 2>&1 || { echo C3 TXN FAILED; tail -5 gpurun_out/c3_txn.log; exit 1; }
tail -1 gpurun_out/c3_txn.log | cut -c1-300
timeout -k 10 500 python3 -u tools/c3_adversarial.py --shape packed --schedules ${C3_SCHED:-pool,uniform,quad} > gpurun_out/c3_packed.log 2>&1 || { echo C3 PACKED FAILED; tail -5 gpurun_out/c3_packed.log; exit 1; }
tail -1 gpurun_out/c3_packed.log | cut -c1-300
