#!/bin/bash
# Round 4: PMC passes over the per-signature path (one signature and a
# 64-signature group commit: fd_k_front + fd_k_dsm_oct) and the quad at
# 4,096 on the final kernels, summarised by tools/pmc4_summary.py.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc_oct
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_THREAD_CYCLES_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_IFETCH"
run() {  # name driver-args counters...
  local name=$1 args=$2; shift 2
  timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o run -- python3 $args > $OUT/$name.txt 2>&1 || { echo "PMC $name FAILED"; tail -5 $OUT/$name.txt; return 1; }
  echo "pass $name ok"
}
( cd $R && timeout -k 10 300 python3 -u -m pytest tests/test_gpu_host.py -m gpu -x -q --timeout 120 --timeout-method thread -k tiny > $R/gpurun_out/pytest_tiny.log 2>&1 ) || { echo TINY FAILED; tail -30 $R/gpurun_out/pytest_tiny.log; exit 1; }
tail -2 $R/gpurun_out/pytest_tiny.log
for cfg in "oct 1" "oct 64" "quad 4096"; do
  set -- $cfg
  run lat_${1}_${2}_p1 "$R/tools/pmc_ring.py $1 $2" $P1 || exit 1
  run lat_${1}_${2}_p2 "$R/tools/pmc_ring.py $1 $2" $P2 || exit 1
done
cd $R
python3 tools/pmc4_summary.py gpurun_out/pmc_oct gpurun_out/pmc_oct.json | cut -c1-400
