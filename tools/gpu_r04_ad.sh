#!/bin/bash
# Round 4, session AD: the front end's per-wave stamps on the final kernels
# (-DFD_FRONT_STAMPS build): a lone signature, a 32-signature group commit
# (both with S's digits recoded ahead) and a lone 4,096 batch.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/front_tail_final.jsonl
for n in 1 32 4096; do
  FD_ED25519_LIB=$PWD/firedancer_amd/variants/lib_fstamps.so timeout -k 10 120 python3 -u tools/front_lone.py 50 $n >> gpurun_out/front_tail_final.jsonl 2> gpurun_out/front_tail_final.err || { echo FRONT FAILED; tail -20 gpurun_out/front_tail_final.err; exit 1; }
done
cut -c1-900 gpurun_out/front_tail_final.jsonl
