#!/bin/bash
# Round 4 host-side measurements on the GPU box's CPU share: the verify
# tile's host feed at C5 shape (tools/tile_host_prof.cpp; memcpy = the
# round-3 frag copy, copy = streaming stores + burst prefetch, inplace =
# no copy), then the native per-signature drop-in benchmark
# (tools/per_sig_threads.cpp, needs the GPU).
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/tile_host_prof.jsonl
: > $O
for r in 1 2 3; do
  for m in memcpy copy inplace; do
    B=tools/build/tile_host_prof; [ $m = memcpy ] && B=tools/build/tile_host_prof_memcpy
    M=$m; [ $m = memcpy ] && M=copy
    for bs in 65536 4096; do
      timeout -k 5 60 $B 65536 2 $bs $M | sed "s/^{/{\"build\": \"$m\", /" >> $O || { echo HOSTPROF FAILED; exit 1; }
    done
  done
done
timeout -k 5 60 tools/build/tile_host_prof_stamps 65536 2 65536 copy | sed 's/^{/{"build": "stamps", /' >> $O
timeout -k 5 60 tools/build/tile_host_prof_stamps 65536 2 65536 inplace | sed 's/^{/{"build": "stamps", /' >> $O
cat $O
timeout -k 10 200 tools/build/per_sig_threads 2000 > gpurun_out/per_sig_threads.jsonl 2> gpurun_out/per_sig_threads.err || { echo PERSIG FAILED; tail gpurun_out/per_sig_threads.err; exit 1; }
cat gpurun_out/per_sig_threads.jsonl
