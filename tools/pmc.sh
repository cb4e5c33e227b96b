#!/bin/bash
# PMC passes over a short bench run (one pass per counter group; FETCH_SIZE
# and WRITE_SIZE each need their own pass on gfx950).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc
mkdir -p $OUT
ARGS="--steps 3 --warmup 1 --no-cpu --no-latency"
run() {  # name counters...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o run -- python3 $R/bench.py $ARGS > $OUT/$name.log 2>&1 || { echo "PMC $name FAILED"; tail -5 $OUT/$name.log; return 1; }
  echo "pass $name ok"
}
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
run sq   SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT && \
run sq2  SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS && \
run fetch FETCH_SIZE && \
run write WRITE_SIZE && \
run l2 TCC_HIT_sum TCC_MISS_sum
