# the ring's H2D by SDMA (default) vs blit kernels (HSA_ENABLE_SDMA=0, set per process)
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/ab_sdma.jsonl
for R in 1 2; do for S in 1 0; do for W in 6 1; do
  HSA_ENABLE_SDMA=$S timeout -k 10 120 python3 -u tools/ring_trace.py --window $W --batches 3000 > gpurun_out/sdma.tmp 2> gpurun_out/sdma.err || { tail -20 gpurun_out/sdma.err; exit 1; }
  echo "{\"sdma\": $S, \"round\": $R, \"res\": $(cat gpurun_out/sdma.tmp)}" >> gpurun_out/ab_sdma.jsonl
done; done; done
cat gpurun_out/ab_sdma.jsonl
