#!/bin/bash
# Round 4, session C: throughput vs signatures per HBM-resident launch
# (the pool's ramp and last round amortised over more waves), two A/B rounds.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/step_ab.txt
for r in 1 2; do
  for B in 256 512; do
    timeout -k 10 300 python3 -u bench.py --no-cpu --no-latency --step-batches $B --steps 10 > gpurun_out/sw.json 2> gpurun_out/sw.err || { echo "FAILED $B"; tail -20 gpurun_out/sw.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/sw.json')); k=d['roofline']['per_kernel']
print('$B', round(d['value']/1e6,3), round(d['ms_per_step'],3), 'pool_frac', round(d['roofline']['frac'],4), ' '.join('%s=%.4f'%(n[5:],v['ms']) for n,v in k.items()), d['codes_ok'])" | tee -a gpurun_out/step_ab.txt
  done
done
