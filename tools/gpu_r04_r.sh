#!/bin/bash
# Round 4, session R: the C5 tile stream at small batches with a deeper
# engine ring (depth 8, as the C2 ring legs) -- copy, in place, and one
# multi-engine in-place tile over two engines.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/tile_c5_r.jsonl
for m in "" "--inplace" "--inplace --multi --tiles 2"; do
  for b in 4096 16384; do
    for d in 4 8; do
      timeout -k 10 120 python3 -u tools/bench_tile.py --sigs 524288 --batch $b --depth $d --seconds 6 --tiles 1 $m >> gpurun_out/tile_c5_r.jsonl 2>> gpurun_out/tile_c5_r.err || { echo TILE FAILED; tail -20 gpurun_out/tile_c5_r.err; exit 1; }
    done
  done
done
python3 -c "
import json
for l in open('gpurun_out/tile_c5_r.jsonl'):
    d=json.loads(l); print(d['batch_sigs'], 'depth', d['depth'], 'inplace' if d['inplace'] else 'copy', 'multi' if d['multi_engine_tile'] else '', round(d['value']/1e6,2), 'M/s')
"
