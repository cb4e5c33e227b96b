#!/bin/bash
# kernel-trace stats + two PMC passes over tools/time_kernels.py (experiments)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pk
mkdir -p $OUT
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 $R/tools/time_kernels.py > $OUT/kt.log 2>&1 || { echo KT FAILED; tail -5 $OUT/kt.log; exit 1; }
cat $(find $OUT/kt -name "*kernel_stats.csv" | head -1) | cut -d, -f1-4 | head -12
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq -o run -- python3 $R/tools/time_kernels.py > $OUT/sq.log 2>&1 || { echo SQ FAILED; tail -5 $OUT/sq.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH --output-format csv -d $OUT/sq2 -o run -- python3 $R/tools/time_kernels.py > $OUT/sq2.log 2>&1 || { echo SQ2 FAILED; tail -5 $OUT/sq2.log; exit 1; }
python3 - <<PY
import csv,glob,collections
for d in ("sq","sq2"):
    f=glob.glob("$OUT/%s/**/*counter_collection.csv"%d, recursive=True)
    if not f: print("no csv",d); continue
    acc=collections.defaultdict(lambda: collections.defaultdict(float)); cnt=collections.Counter()
    for r in csv.DictReader(open(f[0])):
        k=r.get("Kernel_Name",""); 
        if not k.startswith("fd_k"): continue
        acc[k][r["Counter_Name"]]+=float(r["Counter_Value"])
    for k,v in acc.items(): print(d,k,{a:round(b/13) for a,b in v.items()})
PY
