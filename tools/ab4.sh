#!/bin/bash
# A/B/C/D timing of library variants built under firedancer_amd/exp/
set -o pipefail
mkdir -p gpurun_out
for L in "$@"; do
  FD_ED25519_LIB=$L timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_pytest.log 2>&1 || { echo "TESTS FAILED $L"; tail -30 gpurun_out/ab_pytest.log; exit 1; }
  echo "tests ok $L: $(tail -1 gpurun_out/ab_pytest.log)"
done
for r in 1 2; do
  for L in "$@"; do
    FD_ED25519_LIB=$L timeout -k 10 200 python3 -u bench.py --no-cpu --no-latency > gpurun_out/ab.json 2> gpurun_out/ab.err || { echo "FAILED $L"; tail -20 gpurun_out/ab.err; exit 1; }
    python3 -c "
import json,sys; d=json.load(open('gpurun_out/ab.json')); k=d['roofline']['per_kernel']
print('$L', round(d['value']/1e6,3), ' '.join('%s=%.4f'%(n[5:],v['ms']) for n,v in k.items()))"
  done
done
