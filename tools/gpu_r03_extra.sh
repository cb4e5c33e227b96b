#!/bin/bash
# round-3 evidence: PMC passes over the bench (-> profiles pmc summary),
# the C1/C4 configs, and a per-signature drop-in latency sample
set -o pipefail
mkdir -p gpurun_out
bash tools/pmc.sh > gpurun_out/pmc.txt 2>&1 || { echo PMC FAILED; tail -20 gpurun_out/pmc.txt; exit 1; }
tail -6 gpurun_out/pmc.txt
python3 tools/pmc_summary.py gpurun_out/pmc gpurun_out/pmc_traffic.json 1048576 > gpurun_out/pmc_summary.txt 2>&1 || { echo SUMMARY FAILED; tail -20 gpurun_out/pmc_summary.txt; exit 1; }
timeout -k 10 400 python3 -u tools/bench_configs.py > gpurun_out/configs.jsonl 2> gpurun_out/configs.err || { echo CONFIGS FAILED; tail -30 gpurun_out/configs.err; exit 1; }
cat gpurun_out/configs.jsonl | cut -c1-400
timeout -k 10 200 python3 -u tools/per_sig_threads.py > gpurun_out/per_sig.jsonl 2> gpurun_out/per_sig.err || { echo PERSIG FAILED; tail -20 gpurun_out/per_sig.err; exit 1; }
cat gpurun_out/per_sig.jsonl | cut -c1-300
