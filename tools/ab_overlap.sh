#!/bin/bash
# A/B of the device-resident pipeline on one box: serial launches, overlapped
# launches with the DSM stream at default priority, overlapped with the DSM
# stream at high priority (the default); 2 rounds each, bench.py throughput
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for cfg in "FD_BENCH_SERIAL=1" "FD_ED25519_GPU_DSM_PRIO=0" "FD_BENCH_NONE=1"; do
    env $cfg timeout -k 10 200 python3 -u bench.py --no-cpu --no-latency > gpurun_out/abo.json 2> gpurun_out/abo.err || { echo "FAILED $cfg"; tail -5 gpurun_out/abo.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/abo.json')); k=d['roofline']['per_kernel']
print('$cfg', round(d['value']/1e6,3), round(d['ms_per_step'],3), 'pool_live', round(k['fd_k_dsm_pool']['ms'],3), 'frac', round(d['roofline']['frac'],3))"
  done
done
