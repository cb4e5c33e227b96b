#!/bin/bash
# one PMC pass over tools/time_kernels.py for a library variant:
#   tools/pmc_lib.sh <lib.so> <tag> COUNTER...
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; LIB=$1; TAG=$2; shift 2
OUT=$R/gpurun_out/pl/$TAG
mkdir -p $OUT
FD_ED25519_LIB=$R/$LIB timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $OUT -o run -- python3 $R/tools/time_kernels.py > $OUT.log 2>&1 || { echo "PMC $TAG FAILED"; tail -5 $OUT.log; exit 1; }
python3 - <<PY
import csv,glob,collections
f=glob.glob("$OUT/**/*counter_collection.csv", recursive=True)
acc=collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(f[0])):
    k=r.get("Kernel_Name","")
    if k.startswith("fd_k_dsm_pool"): acc[k][r["Counter_Name"]]+=float(r["Counter_Value"])
for k,v in acc.items(): print("$TAG",k,{a:round(b/13) for a,b in v.items()})
PY
