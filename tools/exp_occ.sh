#!/bin/bash
# DSM occupancy / launch-size experiment: per-kernel times for variants.
set -o pipefail
mkdir -p gpurun_out/exp
run() { # name lib stepbatches
  FD_ED25519_LIB=$2 timeout -k 10 120 python3 -u bench.py --no-cpu --no-latency --steps 10 --warmup 2 --step-batches $3 > gpurun_out/exp/$1.json 2>gpurun_out/exp/$1.err || { echo "$1 FAILED"; tail -5 gpurun_out/exp/$1.err; return 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/exp/$1.json'));print('$1', round(d['value']/1e6,2), {k:round(v['ms'],3) for k,v in d['roofline']['per_kernel'].items()})"
}
L=$PWD/firedancer_amd
run w3_s48 $L/libfd_ed25519_gpu.so 48 && run w3_s64 $L/libfd_ed25519_gpu.so 64 && run w3_s96 $L/libfd_ed25519_gpu.so 96 && \
run w2_s32 $L/exp/lib_w2.so 32 && run w2_s64 $L/exp/lib_w2.so 64 && run w4_s64 $L/exp/lib_w4.so 64 && run w4_s128 $L/exp/lib_w4.so 128
