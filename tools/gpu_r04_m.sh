#!/bin/bash
# Round 4, session M: in-place tile batches across the frag ring's wrap
# (two DMA pieces): the tile / engine-host GPU tests, then the C5 tile
# stream copy vs in place at 65536 and 262144 signatures per batch.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_verify_tile.py tests/test_verify_tile_task.py tests/test_gpu_host.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_tile.log 2>&1 || { echo TILE TESTS FAILED; grep -E "FAILED|Error" gpurun_out/pytest_tile.log | head -30; tail -40 gpurun_out/pytest_tile.log; exit 1; }
tail -3 gpurun_out/pytest_tile.log
: > gpurun_out/tile_c5_m.jsonl
for m in "" "--inplace" "--inplace --multi --tiles 2"; do
  for b in 65536 262144; do
    timeout -k 10 120 python3 -u tools/bench_tile.py --sigs 524288 --batch $b --seconds 8 --tiles 1 $m >> gpurun_out/tile_c5_m.jsonl 2>> gpurun_out/tile_c5_m.err || { echo TILE FAILED; tail -20 gpurun_out/tile_c5_m.err; exit 1; }
  done
done
python3 -c "
import json
for l in open('gpurun_out/tile_c5_m.jsonl'):
    d=json.loads(l); print(d['batch_sigs'], 'inplace' if d['inplace'] else 'copy', 'multi' if d['multi_engine_tile'] else '', round(d['value']/1e6,2), 'M/s batches', d['diag'].get('BATCH_CNT'))
"
