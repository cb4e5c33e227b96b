#!/bin/bash
# Round 4, session V (experiment): is the lone quad-DSM wave bound by its
# instruction count?  50 and 100 extra independent full-rate VALU per
# step (-DFD_QUAD_PAD, variants/lib_qpad*.so) against the product
# library: loop cycles per wave of lone 4,096-signature batches.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/qpad.jsonl
for r in 1 2; do
  for v in prod qpad50 qpad100; do
    L=""; [ $v != prod ] && L=$GRAFT_REPO_ROOT/firedancer_amd/variants/lib_$v.so
    FD_ED25519_LIB=$L timeout -k 10 120 python3 -u tools/oct_clock.py 100 2>> gpurun_out/qpad.err | sed "s/^{/{\"lib\": \"$v\", \"round\": $r, /" >> gpurun_out/qpad.jsonl || { echo CLOCK FAILED; tail -20 gpurun_out/qpad.err; exit 1; }
  done
done
python3 -c "
import json
for l in open('gpurun_out/qpad.jsonl'):
    d=json.loads(l); print(d['lib'], d['round'], 'quad', d['quad_n4096']['loop_cycles_per_wave'], round(d['quad_n4096']['ghz'],3))
"
