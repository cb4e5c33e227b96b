#!/bin/bash
# A/B of the host round trip (depth-1 and depth-3 latency over 4096-signature
# C2 batches) between two library builds: tools/lat_ab.sh libA.so libB.so [rounds]
set -o pipefail
A=$1; B=$2; R=${3:-2}
mkdir -p gpurun_out
for r in $(seq 1 $R); do
  for L in $A $B; do
    FD_ED25519_LIB=$L timeout -k 10 200 python3 -u bench.py --no-cpu --steps 2 --warmup 1 --latency-batches 4000 > gpurun_out/lab.json 2> gpurun_out/lab.err || { echo "FAILED $L"; tail -20 gpurun_out/lab.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/lab.json')); l=d['latency']; l1=l['depth1']
print('$L', 'd3 p50 %.3f p99 %.3f | d1 p50 %.3f p99 %.3f'%(l['p50_ms'],l['p99_ms'],l1['p50_ms'],l1['p99_ms']))"
  done
done
