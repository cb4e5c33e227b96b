#!/bin/bash
# host-hop stamps (push -> pick -> submit) on the C2 ring legs of bench.py
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_host.py tests/test_gpu_configs.py -m gpu -x -q --timeout 150 --timeout-method thread -k "feeder or synth or ring" > gpurun_out/pytest_hop.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/pytest_hop.log; exit 1; }
tail -2 gpurun_out/pytest_hop.log
timeout -k 10 400 python3 -u bench.py --no-cpu > gpurun_out/bench_hop.json 2> gpurun_out/bench_hop.err || { echo BENCH FAILED; tail -20 gpurun_out/bench_hop.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/bench_hop.json')); L=d['latency']
for k,v in [('w6',L)]+[(k,L[k]) for k in ('throughput_point','lower_latency_point','depth1','paced_40M')]:
    print(k, round(v['pcie_inclusive_verifies_per_s']/1e6,2), {x: round(v[x],4) for x in ('p50_ms','p99_ms','push_to_pick_p50_ms','push_to_pick_p99_ms','pick_to_submit_p50_ms','pick_to_submit_p99_ms','submit_to_done_p99_ms')})
print('value', d['value']/1e6)
"
