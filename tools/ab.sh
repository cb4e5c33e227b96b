#!/bin/bash
# A/B timing of library variants: tools/ab.sh libA.so libB.so [rounds]
# Alternates short bench runs (no CPU leg) and prints the per-kernel ms.
set -o pipefail
A=$1; B=$2; R=${3:-3}
mkdir -p gpurun_out
for r in $(seq 1 $R); do
  for L in $A $B; do
    FD_ED25519_LIB=$L timeout -k 10 200 python3 -u bench.py --no-cpu --no-latency > gpurun_out/ab.json 2> gpurun_out/ab.err || { echo "FAILED $L"; tail -20 gpurun_out/ab.err; exit 1; }
    python3 -c "
import json,sys; d=json.load(open('gpurun_out/ab.json')); k=d['roofline']['per_kernel']
print('$L', round(d['value']/1e6,3), ' '.join('%s=%.4f'%(n[5:],v['ms']) for n,v in k.items()))"
  done
done
