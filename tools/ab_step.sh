#!/bin/bash
# bench.py throughput at several step sizes (batches of 4096 per fused launch), interleaved
# usage: tools/ab_step.sh 256 512 256 512
set -o pipefail
mkdir -p gpurun_out
for sb in "$@"; do
  timeout -k 10 300 python3 -u bench.py --no-cpu --no-latency --step-batches $sb --steps 10 > gpurun_out/bsb.json 2> gpurun_out/bsb.err || { echo "FAILED $sb"; tail -5 gpurun_out/bsb.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/bsb.json'))
print($sb, round(d['value']/1e6,2), round(d['ms_per_step'],2), d['codes_ok'], round(d['roofline']['frac'],3))"
done
