#!/bin/bash
# Round 4, session T: the quad DSM with independent column chains
# (FD_QUAD_ILP=1, variants/lib_qilp.so) against the absorbed chain (the
# product library): loop cycles per wave of lone 4,096-signature batches,
# two rounds.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/qilp_ab.jsonl
for r in 1 2; do
  for v in absorbed ilp; do
    L=""; [ $v = ilp ] && L=$GRAFT_REPO_ROOT/firedancer_amd/variants/lib_qilp.so
    FD_ED25519_LIB=$L timeout -k 10 120 python3 -u tools/oct_clock.py 200 2>> gpurun_out/qilp_ab.err | sed "s/^{/{\"lib\": \"$v\", \"round\": $r, /" >> gpurun_out/qilp_ab.jsonl || { echo CLOCK FAILED; tail -20 gpurun_out/qilp_ab.err; exit 1; }
  done
done
python3 -c "
import json
for l in open('gpurun_out/qilp_ab.jsonl'):
    d=json.loads(l); print(d['lib'], d['round'], 'quad', d['quad_n4096']['loop_cycles_per_wave'], round(d['quad_n4096']['ghz'],3), d['quad_n4096']['call_p50_ms'], 'oct', d['oct_n1']['loop_cycles_per_wave'])
"
