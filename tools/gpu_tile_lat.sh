#!/bin/bash
# verify tile: multi-engine GPU tests, then the C5 tsorig -> tspub latency
# curve over batch sizes (one tile per GPU, and one multi-engine tile on 2
# engines of this GPU), PCIe included
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_verify_tile.py tests/test_verify_tile_task.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/pytest_tile.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/pytest_tile.log; exit 1; }
tail -3 gpurun_out/pytest_tile.log
timeout -k 10 400 python3 -u tools/bench_tile.py --curve 4096,16384,65536,262144 --sigs 524288 --seconds 8 --tiles 2 > gpurun_out/tile_lat_curve.jsonl 2> gpurun_out/tile_lat.err || { echo CURVE FAILED; tail -20 gpurun_out/tile_lat.err; exit 1; }
timeout -k 10 200 python3 -u tools/bench_tile.py --curve 16384,65536 --sigs 524288 --seconds 8 --tiles 2 --multi >> gpurun_out/tile_lat_curve.jsonl 2>> gpurun_out/tile_lat.err || { echo MULTI FAILED; tail -20 gpurun_out/tile_lat.err; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/tile_lat_curve.jsonl'):
    d=json.loads(l); L=d['latency_tsorig_to_tspub']
    print(d['batch_sigs'], 'multi' if d['multi_engine_tile'] else 'tiles', round(d['value']/1e6,2), 'M/s', {k: round(v,3) if isinstance(v,float) else v for k,v in L.items()})
"
