#!/bin/bash
# A/B of library variants on the C2 ring (tools/ring_sweep.py), interleaved,
# 2 rounds.  usage: tools/ab_ring.sh "<ring_sweep args>" lib1.so lib2.so ...
set -o pipefail
mkdir -p gpurun_out
ARGS=$1; shift
for r in 1 2; do
  for L in "$@"; do
    FD_ED25519_LIB=$L timeout -k 10 300 python3 -u tools/ring_sweep.py $ARGS 2>/dev/null | python3 -c "
import json, sys
for l in sys.stdin:
    d = json.loads(l)
    print('$L', d['ring_depth'], d['window'], round(d['pcie_inclusive_verifies_per_s'] / 1e6, 2), round(d['p50_ms'], 3), round(d['p99_ms'], 3), round(d['p999_ms'], 3))
" || { echo "FAILED $L"; exit 1; }
  done
done
