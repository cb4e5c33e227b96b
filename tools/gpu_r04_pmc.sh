#!/bin/bash
# Round 4: PMC passes over the latency schedule's kernels (tools/pmc_ring.py:
# lone device-resident batches; quad and quad2 at one and two waves per SIMD)
# and over the throughput step (bench.py), then the quad-DSM stamps build
# lone and under the ring (tools/quad_stamps.py).  Each GPU step has its own
# limit; the chain stops at the first failure.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc4
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_THREAD_CYCLES_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_IFETCH"
P3="SQ_WAIT_INST_LDS SQ_IFETCH SQ_IFETCH_LEVEL SQ_INST_CYCLES_VMEM_RD SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM"
run() {  # name driver-args counters...
  local name=$1 args=$2; shift 2
  timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o run -- python3 $args > $OUT/$name.txt 2>&1 || { echo "PMC $name FAILED"; tail -5 $OUT/$name.txt; return 1; }
  echo "pass $name ok"
}
for cfg in "quad 4096" "quad 16384"; do
  set -- $cfg
  run lat_${1}_${2}_p1 "$R/tools/pmc_ring.py $1 $2" $P1 || exit 1
  run lat_${1}_${2}_p2 "$R/tools/pmc_ring.py $1 $2" $P2 || exit 1
done
B="$R/bench.py --steps 3 --warmup 1 --no-cpu --no-latency"
run thr_p1 "$B" $P1 || exit 1
run thr_p3 "$B" $P3 || exit 1
run thr_fetch "$B" FETCH_SIZE || exit 1
run thr_write "$B" WRITE_SIZE || exit 1
cd $R
FD_ED25519_LIB=$R/firedancer_amd/variants/lib_qstamps.so timeout -k 10 240 python3 -u tools/quad_stamps.py 3000 > gpurun_out/quad_stamps.jsonl 2> gpurun_out/quad_stamps.err || { echo STAMPS FAILED; tail -20 gpurun_out/quad_stamps.err; exit 1; }
cat gpurun_out/quad_stamps.jsonl
