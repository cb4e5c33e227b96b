# where the latency front end's time goes: stamps build, lone launches and the ring at 6 / 8 in flight
set -o pipefail
mkdir -p gpurun_out
S=firedancer_amd/variants/lib_stamps.so
FD_ED25519_LIB=$S timeout -k 10 200 python3 -u tools/front_lone.py > gpurun_out/front_split.jsonl 2> gpurun_out/front_split.err || { tail -20 gpurun_out/front_split.err; exit 1; }
for W in 6 8; do
  FD_ED25519_LIB=$S timeout -k 10 200 python3 -u tools/front_stamps.py 8 $W 3000 >> gpurun_out/front_split.jsonl 2>> gpurun_out/front_split.err || { tail -20 gpurun_out/front_split.err; exit 1; }
done
cat gpurun_out/front_split.jsonl
