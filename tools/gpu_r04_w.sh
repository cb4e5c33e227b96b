#!/bin/bash
# Round 4, session W (experiment): is the decompression wave on the lone
# signature's critical path?  The front end with its decomp blocks skipped
# (-DFD_EXP_SKIP_DECOMP, wrong codes, timing only) against the product
# library: single-signature call p50 and the oct loop (unchanged inputs).
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/skipdecomp.jsonl
for r in 1 2; do
  for v in prod skipdecomp; do
    L=""; [ $v != prod ] && L=$GRAFT_REPO_ROOT/firedancer_amd/variants/lib_$v.so
    FD_ED25519_LIB=$L timeout -k 10 120 python3 -u tools/oct_clock.py 400 2>> gpurun_out/skipdecomp.err | sed "s/^{/{\"lib\": \"$v\", \"round\": $r, /" >> gpurun_out/skipdecomp.jsonl || { echo CLOCK FAILED; tail -20 gpurun_out/skipdecomp.err; exit 1; }
  done
done
python3 -c "
import json
for l in open('gpurun_out/skipdecomp.jsonl'):
    d=json.loads(l); print(d['lib'], d['round'], 'oct call p50', round(d['oct_n1']['call_p50_ms']*1e3,1), 'us loop', d['oct_n1']['loop_cycles_per_wave'], 'quad call p50', round(d['quad_n4096']['call_p50_ms']*1e3,1))
"
