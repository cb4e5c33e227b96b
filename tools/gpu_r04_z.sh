#!/bin/bash
# Round 4, session Z (experiment): is the quad step's output mix on its critical
# path?  The mix without its R and S terms (-DFD_QUAD_MIX_PROBE, wrong
# codes, timing only) against the product
# library: loop cycles per wave of lone 4,096-signature batches.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/mixprobe.jsonl
for r in 1 2; do
  for v in prod mixprobe; do
    L=""; [ $v != prod ] && L=$GRAFT_REPO_ROOT/firedancer_amd/variants/lib_$v.so
    FD_ED25519_LIB=$L timeout -k 10 120 python3 -u tools/oct_clock.py 100 2>> gpurun_out/mixprobe.err | sed "s/^{/{\"lib\": \"$v\", \"round\": $r, /" >> gpurun_out/mixprobe.jsonl || { echo CLOCK FAILED; tail -20 gpurun_out/mixprobe.err; exit 1; }
  done
done
python3 -c "
import json
for l in open('gpurun_out/mixprobe.jsonl'):
    d=json.loads(l); print(d['lib'], d['round'], 'quad', d['quad_n4096']['loop_cycles_per_wave'], round(d['quad_n4096']['ghz'],3))
"
