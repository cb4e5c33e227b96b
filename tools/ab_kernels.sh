#!/bin/bash
# per-kernel serial timing (tools/time_kernels.py) of library variants,
# interleaved, 3 rounds; and the fused quad DSM at 4096 signatures
# usage: tools/ab_kernels.sh lib1.so lib2.so ...
set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3; do
  for L in "$@"; do
    FD_ED25519_LIB=$L timeout -k 10 120 python3 -u tools/time_kernels.py 1048576 2>/dev/null || { echo "FAILED $L"; exit 1; }
    FD_ED25519_LIB=$L timeout -k 10 120 python3 -u tools/time_kernels.py 4096 2>/dev/null || { echo "FAILED $L"; exit 1; }
  done
done
