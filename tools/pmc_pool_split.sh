#!/bin/bash
# HBM bytes of fd_k_dsm_pool split into Ai-entry reads and the rest: the
# FETCH_SIZE / WRITE_SIZE passes of tools/pmc.sh on the product library and
# on a diagnostic build whose Ai reads all hit one cached table
# (-DFD_POOL_TRAFFIC_DIAG, variants/libtdiag.so; its codes are wrong)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmcsplit
mkdir -p $OUT
ARGS="--steps 3 --warmup 1 --no-cpu --no-latency"
for V in product diag; do
  if [[ $V == diag ]]; then export FD_ED25519_LIB=$R/firedancer_amd/variants/libtdiag.so; fi
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/$V/fetch -o run -- python3 $R/bench.py $ARGS > $OUT/$V.fetch.log 2>&1 || { echo "FETCH $V FAILED"; tail -5 $OUT/$V.fetch.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/$V/write -o run -- python3 $R/bench.py $ARGS > $OUT/$V.write.log 2>&1 || { echo "WRITE $V FAILED"; tail -5 $OUT/$V.write.log; exit 1; }
done
python3 - <<PY
import csv, glob, collections, json
res = {}
for v in ("product", "diag"):
    for c in ("fetch", "write"):
        f = glob.glob("$OUT/%s/%s/**/*counter_collection.csv" % (v, c), recursive=True)[0]
        acc = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            if r.get("Kernel_Name", "").startswith("fd_k_dsm_pool"):
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, xs in acc.items():
            res["%s_%s" % (v, k)] = sum(xs) / len(xs)
n = 1048576
p = 2 * res["product_FETCH_SIZE"] * 1024 + res["product_WRITE_SIZE"] * 1024
d = 2 * res["diag_FETCH_SIZE"] * 1024 + res["diag_WRITE_SIZE"] * 1024
print(json.dumps({"raw_kb_per_launch": res, "sigs_per_launch": n,
                  "hbm_bytes_per_sig_product": p / n, "hbm_bytes_per_sig_without_ai_reads": d / n,
                  "ai_entry_bytes_per_sig": (p - d) / n,
                  "note": "hbm = 2*FETCH_SIZE + WRITE_SIZE (KB units, gfx950 16-B/lane fetch correction, tools/pmc_summary.py)"}))
PY
