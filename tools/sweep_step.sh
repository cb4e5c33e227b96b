#!/bin/bash
# bench.py throughput vs signatures per launch (4096-sig batches per step)
set -o pipefail
mkdir -p gpurun_out
for B in "$@"; do
  timeout -k 10 300 python3 -u bench.py --no-cpu --no-latency --step-batches $B --steps 10 > gpurun_out/sw.json 2> gpurun_out/sw.err || { echo "FAILED $B"; tail -20 gpurun_out/sw.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/sw.json')); k=d['roofline']['per_kernel']
print('$B', round(d['value']/1e6,3), ' '.join('%s=%.4f'%(n[5:],v['ms']) for n,v in k.items()))"
done
