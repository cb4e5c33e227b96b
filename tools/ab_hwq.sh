#!/bin/bash
# Ring sweep under different GPU_MAX_HW_QUEUES values (HIP hardware queues
# per process; the box's default is 4): tools/ab_hwq.sh "<ring_sweep args>" 4 8 16
set -o pipefail
mkdir -p gpurun_out
ARGS=$1; shift
for r in 1 2; do
  for Q in "$@"; do
    GPU_MAX_HW_QUEUES=$Q timeout -k 10 300 python3 -u tools/ring_sweep.py $ARGS 2>gpurun_out/hwq.err | python3 -c "
import json, sys
for l in sys.stdin:
    d = json.loads(l)
    print('hwq=$Q', d['ring_depth'], d['window'], round(d['pcie_inclusive_verifies_per_s'] / 1e6, 2), round(d['p50_ms'], 3), round(d['p99_ms'], 3), round(d['p999_ms'], 3))
" || { echo "FAILED $Q"; tail -5 gpurun_out/hwq.err; exit 1; }
  done
done
