#!/bin/bash
# Round 4: the bench's multi-rank path on the final tree, rehearsed with two
# ranks sharing the box's one GPU (FD_BENCH_SHARE_GPU=1: gloo barrier and
# max-over-ranks; the driver runs 1/2/4/8 GPUs with RCCL on a real node).
set -o pipefail
mkdir -p gpurun_out
FD_BENCH_SHARE_GPU=1 timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/bench_n2.json 2> gpurun_out/bench_n2.err || { echo N2 FAILED; tail -30 gpurun_out/bench_n2.err; exit 1; }
cut -c1-600 gpurun_out/bench_n2.json
