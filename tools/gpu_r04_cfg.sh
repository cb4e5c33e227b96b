#!/bin/bash
# Round 4, final kernels: the other BASELINE configs (C1, C4) on one MI355X.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python3 -u tools/bench_configs.py > gpurun_out/configs_final.jsonl 2> gpurun_out/configs_final.err || { echo CONFIGS FAILED; tail -20 gpurun_out/configs_final.err; exit 1; }
cut -c1-700 gpurun_out/configs_final.jsonl
