#!/bin/bash
# Round 4, session AA (A/B): group-commit leaders of fd_ed25519_verify (=
# the default engine's ring depth) 3 (default) vs 6 vs 8, native threads.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/vq_leaders.jsonl
for r in 1 2; do
  for v in 3 6 8; do
    echo "run leaders=$v round=$r" | tee -a gpurun_out/vq_leaders.log
    FD_ED25519_GPU_VQ_LEADERS=$v timeout -k 10 90 stdbuf -oL ./tools/build/per_sig_threads 2000 > gpurun_out/vq_$v.$r.jsonl 2> gpurun_out/vq_leaders.err || { echo PERSIG FAILED rc=$?; tail -20 gpurun_out/vq_leaders.err; cat gpurun_out/vq_$v.$r.jsonl; exit 1; }
    sed "s/^{/{\"leaders\": $v, \"round\": $r, /" gpurun_out/vq_$v.$r.jsonl >> gpurun_out/vq_leaders.jsonl
  done
done
python3 -c "
import json
for l in open('gpurun_out/vq_leaders.jsonl'):
    d=json.loads(l); print(d['leaders'], d['round'], d['threads'], d['calls_per_s'], d['p50_ms'], d['p99_ms'], d['max_ms'])
"
