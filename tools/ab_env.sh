#!/bin/bash
# A/B of engine/bench environment knobs on one box:
#   tools/ab_env.sh ROUNDS "CFG_A" "CFG_B" ...   (CFG = "VAR=val [VAR=val]", "FD_BENCH_NONE=1" for the default)
# Alternates short bench runs (no CPU or latency leg); prints throughput,
# step time, the pool's live ms and the roofline frac.
set -o pipefail
mkdir -p gpurun_out
R=$1; shift
for r in $(seq 1 $R); do
  for cfg in "$@"; do
    env $cfg timeout -k 10 200 python3 -u bench.py --no-cpu --no-latency > gpurun_out/abe.json 2> gpurun_out/abe.err || { echo "FAILED $cfg"; tail -5 gpurun_out/abe.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/abe.json')); k=d['roofline']['per_kernel']
print('$cfg', round(d['value']/1e6,3), round(d['ms_per_step'],3), 'pool_live', round(k['fd_k_dsm_pool']['ms'],3), 'frac', round(d['roofline']['frac'],3), 'ok', d['codes_ok'])"
  done
done
