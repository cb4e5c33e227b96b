#!/bin/bash
# Round 4, session B2 (the tail of session B, whose stamps step met a stale
# diagnostic build): the quad-DSM stamps, the C5 verify-tile stream in the
# copy and in-place modes, then session C (signatures per HBM-resident
# launch, 256 vs 512 batches).  Each GPU step has its own limit; the chain
# stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
FD_ED25519_LIB=$R/firedancer_amd/variants/lib_qstamps.so timeout -k 10 240 python3 -u tools/quad_stamps.py 3000 > gpurun_out/quad_stamps.jsonl 2> gpurun_out/quad_stamps.err || { echo STAMPS FAILED; tail -20 gpurun_out/quad_stamps.err; exit 1; }
cat gpurun_out/quad_stamps.jsonl
: > gpurun_out/tile_c5.jsonl
for m in "" "--inplace" "--inplace --multi --tiles 2"; do
  for b in 4096 65536 262144; do
    timeout -k 10 120 python3 -u tools/bench_tile.py --sigs 524288 --batch $b --seconds 8 --tiles 1 $m >> gpurun_out/tile_c5.jsonl 2>> gpurun_out/tile_c5.err || { echo TILE FAILED; tail -20 gpurun_out/tile_c5.err; exit 1; }
  done
done
cut -c1-400 gpurun_out/tile_c5.jsonl
bash tools/gpu_r04_c.sh
