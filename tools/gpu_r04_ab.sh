#!/bin/bash
# Round 4, session AB: the latency DSMs issue every prologue load before using any
# (status, points, op rows, Bi: one memory round trip instead of several).
# The whole GPU suite (incl. the 10 M corpus under the quad and oct
# schedules), then the A/B of the latency DSMs' loop cycles per wave
# (base = the previous library, variants/lib_base.so), two rounds,
# the per-signature runs and the bench without the CPU leg.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1 || { echo GPU TESTS FAILED; grep -E "FAILED|Error" gpurun_out/pytest_ab.log | head -30; tail -40 gpurun_out/pytest_ab.log; exit 1; }
tail -3 gpurun_out/pytest_ab.log
: > gpurun_out/pro_ab.jsonl
for r in 1 2; do
  for v in base new; do
    L=""; [ $v = base ] && L=$GRAFT_REPO_ROOT/firedancer_amd/variants/lib_base.so
    FD_ED25519_LIB=$L timeout -k 10 120 python3 -u tools/oct_clock.py 300 2>> gpurun_out/pro_ab.err | sed "s/^{/{\"lib\": \"$v\", \"round\": $r, /" >> gpurun_out/pro_ab.jsonl || { echo CLOCK FAILED; tail -20 gpurun_out/pro_ab.err; exit 1; }
  done
done
python3 -c "
import json
for l in open('gpurun_out/pro_ab.jsonl'):
    d=json.loads(l); print(d['lib'], d['round'], 'oct', d['oct_n1']['loop_cycles_per_wave'], d['oct_n1']['call_p50_ms'], 'quad', d['quad_n4096']['loop_cycles_per_wave'], d['quad_n4096']['call_p50_ms'])
"
timeout -k 10 200 ./tools/build/per_sig_threads 2000 > gpurun_out/per_sig_ab.jsonl 2> gpurun_out/per_sig_ab.err || { echo PERSIG FAILED; tail -20 gpurun_out/per_sig_ab.err; exit 1; }
cut -c1-160 gpurun_out/per_sig_ab.jsonl
timeout -k 10 400 python3 -u bench.py --no-cpu > gpurun_out/bench_ab.json 2> gpurun_out/bench_ab.err || { echo BENCH FAILED; tail -30 gpurun_out/bench_ab.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/bench_ab.json')); l=d['latency']
print('value', d['value'], 'frac', d['roofline']['frac'])
print('closed', l['pcie_inclusive_verifies_per_s'], l['p99_ms'], 'w8', l['window8_point']['pcie_inclusive_verifies_per_s'], l['window8_point']['p99_ms'])
print('paced', [(round(p['offered_verifies_per_s']/1e6), round(p['sched_to_done_p99_ms'],3)) for p in l['paced']])
print('depth1', l['depth1']['p50_ms'], l['depth1']['p99_ms'])
"
