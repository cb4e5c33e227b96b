#!/bin/bash
# per-kernel timing of each library variant given (tools/time_kernels.py)
set -o pipefail
mkdir -p gpurun_out
for L in "$@"; do
  FD_ED25519_LIB=$L timeout -k 10 200 python3 -u tools/time_kernels.py 2> gpurun_out/tv.err || { echo "FAILED $L"; tail -20 gpurun_out/tv.err; exit 1; }
done
