#!/bin/bash
# C5 verify-tile stream (two tiles, 262144-signature batches, 30 s) and the
# bench's N=2 torchrun path rehearsed with two ranks sharing the one GPU.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python3 -u tools/bench_tile.py --seconds 30 --tiles 2 --batch 262144 > gpurun_out/bench_tile_c5.json 2> gpurun_out/bench_tile.err || { echo TILE BENCH FAILED; tail -30 gpurun_out/bench_tile.err; exit 1; }
cut -c1-400 gpurun_out/bench_tile_c5.json
FD_BENCH_SHARE_GPU=1 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/bench_n2.json 2> gpurun_out/bench_n2.err || { echo N2 FAILED; tail -30 gpurun_out/bench_n2.err; exit 1; }
tail -1 gpurun_out/bench_n2.json | cut -c1-300
