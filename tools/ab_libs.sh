#!/bin/bash
# A/B of library variants (firedancer_amd/variants/*.so, experiments only) on
# one box: bench.py throughput (pipelined, HBM-resident), 2 rounds each,
# interleaved.  usage: tools/ab_libs.sh lib1.so lib2.so ...
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for L in "$@"; do
    FD_ED25519_LIB=$L timeout -k 10 200 python3 -u bench.py --no-cpu --no-latency --unique 262144 > gpurun_out/abl.json 2> gpurun_out/abl.err || { echo "FAILED $L"; tail -5 gpurun_out/abl.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/abl.json')); k=d['roofline']['per_kernel']
print('$L', round(d['value']/1e6,3), round(d['ms_per_step'],3), 'ok', d['all_accepted'], ' '.join('%s %.3f/%.3f' % (n[5:], v['ms'], v['ms_serial']) for n, v in k.items()))"
  done
done
