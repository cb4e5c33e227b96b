#!/usr/bin/env python3
"""Summarise the rocprofv3 --pmc passes of tools/pmc.sh into
profiles/pmc_traffic.json (read by bench.py for roofline.traffic).

Per kernel, averaged over its dispatches:
  FETCH_SIZE / WRITE_SIZE (KB, rocprofv3 units) -> bytes per launch.
    MI355X_MICROARCH.md (HBM, gfx950): FETCH_SIZE reports 1/2 of the
    bytes of wide (16 B/lane) reads; WRITE_SIZE is exact for 16 B/lane
    stores.  The engine's dominant reads are 16 B/lane (Ai table entries,
    descriptors), so hbm_bytes_per_launch = 2*FETCH + WRITE; the raw
    counters are kept beside it.
  SQ counters -> VALU wave-instructions per signature, VALU issue rate
    (wave-instructions per SIMD-cycle), effective clock, wait fractions.

usage: pmc_summary.py <gpurun_out/pmc> <out.json> <sigs_per_launch>
The device code the passes ran is named by <gpurun_out/pmc>/kernels.id
(fd_ed25519_gpu_kernels_id, written by tools/gpu.sh pmcthr); bench.py uses
the summary only while that id equals the loaded library's.
"""
import collections
import csv
import json
import os
import sys

SIMDS = 256 * 4
XCDS = 8


def load(d):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in sorted(os.listdir(d)):
        f = os.path.join(d, p, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if k.startswith("fd_k"):
                agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in agg.items()}


def main():
    src, dst, n = sys.argv[1], sys.argv[2], int(sys.argv[3])
    raw = load(src)
    kf = os.path.join(src, "kernels.id")
    kid = open(kf).read().split()[0] if os.path.exists(kf) else None
    out = {"sigs_per_launch": n, "kernels_id": kid, "source": "tools/gpu.sh pmcthr (rocprofv3 --pmc, one pass per group)",
           "correction": "hbm_bytes = 2*FETCH_SIZE + WRITE_SIZE (gfx950 FETCH_SIZE halves 16 B/lane reads)",
           "kernels": {}}
    for k, c in sorted(raw.items()):
        e = {"raw": c}
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            fb, wb = c["FETCH_SIZE"] * 1024, c["WRITE_SIZE"] * 1024
            e["fetch_bytes_raw"] = fb
            e["write_bytes"] = wb
            e["hbm_bytes_per_launch"] = 2 * fb + wb
            e["hbm_bytes_per_sig"] = (2 * fb + wb) / n
        if "SQ_INSTS_VALU" in c and "GRBM_GUI_ACTIVE" in c:
            cyc = c["GRBM_GUI_ACTIVE"] / XCDS
            e["valu_wave_insts_per_sig"] = c["SQ_INSTS_VALU"] * 64 / n
            e["valu_issue_per_simd_cycle"] = c["SQ_INSTS_VALU"] / SIMDS / cyc
            wc = c.get("SQ_WAVE_CYCLES")
            if wc:
                e["wait_any_frac"] = c.get("SQ_WAIT_ANY", 0) / wc
                e["wait_inst_any_frac"] = c.get("SQ_WAIT_INST_ANY", 0) / wc
                e["active_inst_any_frac"] = c.get("SQ_ACTIVE_INST_ANY", 0) / wc
        if "TCC_HIT_sum" in c:
            e["l2_hit_rate"] = c["TCC_HIT_sum"] / max(1.0, c["TCC_HIT_sum"] + c["TCC_MISS_sum"])
        out["kernels"][k] = e
    json.dump(out, open(dst, "w"), indent=1)
    for k, e in out["kernels"].items():
        print(k, {x: (round(y, 4) if isinstance(y, float) else y) for x, y in e.items() if x != "raw"})


if __name__ == "__main__":
    main()
