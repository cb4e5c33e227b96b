#!/usr/bin/env python3
"""Summarise the round-4 PMC passes (tools/gpu_r04_pmc.sh) into one JSON:
per run and kernel, counters averaged over its dispatches plus derived
rates.  Units (MI355X_MICROARCH.md, 'Per-instruction cycle constants'):
SQ_WAVE_CYCLES, SQ_WAIT_*, SQ_ACTIVE_INST_*, SQ_BUSY_CYCLES count in
quad-cycles (x4 = shader cycles); GRBM_GUI_ACTIVE is summed over the 8
XCDs, so the effective clock is GRBM_GUI_ACTIVE / 8 / dispatch time (it
reads high on dispatches shorter than ~0.3 ms); FETCH_SIZE / WRITE_SIZE in
KB, gfx950 FETCH_SIZE halving 16-byte-per-lane reads (x2 for those).

Derived (per dispatch of the kernel):
  valu_per_wave          SQ_INSTS_VALU / SQ_WAVES
  wave_cycles            4 SQ_WAVE_CYCLES / SQ_WAVES (a wave's lifetime, shader cycles)
  cycles_per_valu        wave_cycles / valu_per_wave (one wave's own issue pace)
  valu_issue_per_simd_cycle  SQ_INSTS_VALU / (SIMDs holding waves x dispatch cycles),
                         for the lone-batch runs where each wave has a SIMD to itself
  *_frac                 a wait / active counter / SQ_WAVE_CYCLES

usage: pmc4_summary.py <gpurun_out/pmc4> <out.json>"""
import collections
import csv
import json
import os
import sys

XCDS = 8


def load(path):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    seen = set()
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        if not k.startswith("fd_k"):
            continue
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        key = (k, r["Dispatch_Id"])
        if key not in seen:
            seen.add(key)
            dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    return {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in agg.items()}, \
           {k: sum(v) / len(v) for k, v in dur.items()}


def derive(c, t, sigs):
    e = {"dispatch_ms": t * 1e3}
    w = c.get("SQ_WAVES")
    if w:
        e["waves"] = w
        if "SQ_INSTS_VALU" in c:
            e["valu_per_wave"] = c["SQ_INSTS_VALU"] / w
            e["valu_lane_instr_per_sig"] = c["SQ_INSTS_VALU"] * 64 / sigs if sigs else None
        if "SQ_WAVE_CYCLES" in c:
            e["wave_cycles"] = 4 * c["SQ_WAVE_CYCLES"] / w
            if "valu_per_wave" in e:
                e["cycles_per_valu"] = e["wave_cycles"] / e["valu_per_wave"]
    if "GRBM_GUI_ACTIVE" in c and t > 0:
        e["effective_clock_ghz"] = c["GRBM_GUI_ACTIVE"] / XCDS / t * 1e-9
    wc = c.get("SQ_WAVE_CYCLES")
    if wc:
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_WAIT_INST_LDS",
                  "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VMEM", "SQ_INST_LEVEL_VMEM", "SQ_INST_LEVEL_LDS", "SQ_IFETCH_LEVEL"):
            if k in c:
                e[k.lower() + "_frac"] = c[k] / wc
    if "FETCH_SIZE" in c:
        e["fetch_kb_raw"] = c["FETCH_SIZE"]
        if sigs:
            e["fetch_bytes_per_sig_x2"] = 2 * c["FETCH_SIZE"] * 1024 / sigs
    if "WRITE_SIZE" in c:
        e["write_kb"] = c["WRITE_SIZE"]
        if sigs:
            e["write_bytes_per_sig"] = c["WRITE_SIZE"] * 1024 / sigs
    return e


def main():
    src, dst = sys.argv[1], sys.argv[2]
    out = {"source": "tools/gpu_r04_pmc.sh (rocprofv3 --pmc, one pass per counter group; dispatches serialised)",
           "units": __doc__.split("usage:")[0].strip(), "runs": {}}
    for name in sorted(os.listdir(src)):
        f = os.path.join(src, name, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        sigs = None
        if name.startswith("lat_"):
            sigs = int(name.split("_")[2])
        elif name.startswith("thr_"):
            sigs = 1 << 20
        raw, dur = load(f)
        out["runs"][name] = {k: {"raw": raw[k], **derive(raw[k], dur.get(k, 0.0), sigs)} for k in raw}
    # the quad DSM: a lone wave's issue pace vs one wave per SIMD everywhere
    json.dump(out, open(dst, "w"), indent=1)
    for run, ks in out["runs"].items():
        for k, e in ks.items():
            print(run, k, {x: (round(y, 4) if isinstance(y, float) else y) for x, y in e.items() if x != "raw"})


if __name__ == "__main__":
    main()
