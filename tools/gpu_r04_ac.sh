#!/bin/bash
# Round 4, session AC: the ring's closed- and open-loop points, the product
# library against the previous one (variants/lib_base.so: before the
# prologue loads were batched), alternating, two rounds, one box.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/ring_ab.jsonl
for r in 1 2; do
  for v in base new; do
    L=""; [ $v = base ] && L=$GRAFT_REPO_ROOT/firedancer_amd/variants/lib_base.so
    echo "run $v $r"
    FD_ED25519_LIB=$L timeout -k 10 240 python3 -u tools/ring_paced.py 4000 2>> gpurun_out/ring_ab.err | sed "s/^{/{\"lib\": \"$v\", \"round\": $r, /" >> gpurun_out/ring_ab.jsonl || { echo RING FAILED; tail -20 gpurun_out/ring_ab.err; exit 1; }
    tail -1 gpurun_out/ring_ab.jsonl | cut -c1-400
  done
done
