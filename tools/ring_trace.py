#!/usr/bin/env python3
"""The C2 ring (bench.py's latency leg: 4,096-signature batches through the
feeder, depth 8, `--window` in flight) for a kernel + memory-copy trace,
then (`--analyze DIR`) the per-batch device timeline from that trace:
per CU group, how the H2D of a batch, its front end and its quad DSM line
up with the batch before it on the same group.

  rocprofv3 --kernel-trace --memory-copy-trace -d OUT -- python3 tools/ring_trace.py --window 6
  python3 tools/ring_trace.py --analyze OUT"""
import argparse
import csv
import glob
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(a):
    import torch  # noqa: F401  (HIP runtime before the engine, as bench.py)
    import bench
    import firedancer_amd as fa
    from firedancer_amd import corpus
    base = corpus.solana_txns(65536, seed=1000, nthreads=16)
    bench.ring_stream(fa, base, 0, 50, 8, window=a.window)
    r = bench.ring_stream(fa, base, 0, a.batches, 8, window=a.window)
    print(json.dumps({k: r[k] for k in ("pcie_inclusive_verifies_per_s", "p50_ms", "p99_ms", "window", "ring_depth")}), flush=True)


def rows(d, pat):
    out = []
    for f in glob.glob(os.path.join(d, "**", pat), recursive=True):
        out += list(csv.DictReader(open(f)))
    return out


def analyze(d):
    ks = rows(d, "*kernel_trace.csv")
    cs = rows(d, "*memory_copy_trace.csv")
    ev = []
    for r in ks:
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get("Queue_Id", ""), r.get("Stream_Id", "")))
    for r in cs:
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "COPY_" + r.get("Direction", "?"), r.get("Queue_Id", ""), r.get("Stream_Id", "")))
    ev.sort()
    names = {}
    for e in ev:
        names.setdefault(e[2][:40], 0)
        names[e[2][:40]] += 1
    # per stream: the sequence of events; a batch = H2D(s) .. front .. dsm .. D2H
    streams = {}
    for e in ev:
        streams.setdefault(e[4], []).append(e)
    per = []
    for sid, es in streams.items():
        cur = None
        for e in es:
            n = e[2]
            if n.startswith("COPY_") and ("HOST_TO_DEVICE" in n.upper() or "H2D" in n.upper()):
                if cur is None or "d2h" in cur:
                    cur = {"stream": sid, "h2d0": e[0], "h2d1": e[1]}
                else:
                    cur["h2d1"] = max(cur["h2d1"], e[1])
            elif "fd_k_front" in n and cur is not None:
                cur["f0"], cur["f1"] = e[0], e[1]
            elif "fd_k_dsm" in n and cur is not None:
                cur["q0"], cur["q1"] = e[0], e[1]
            elif (n.startswith("COPY_") or "copyBuffer" in n) and cur is not None and "q1" in cur:
                # the codes' D2H: an SDMA copy or, small as it is, a blit kernel
                cur["d2h"] = e[1]
                per.append(cur)
                cur = None
    if not per:
        return {"events": names, "batches": 0}
    per.sort(key=lambda b: b["h2d0"])
    us = lambda x: float(np.median(x)) / 1e3
    h2d = [b["h2d1"] - b["h2d0"] for b in per]
    g1 = [b["f0"] - b["h2d1"] for b in per]
    fr = [b["f1"] - b["f0"] for b in per]
    g2 = [b["q0"] - b["f1"] for b in per]
    dsm = [b["q1"] - b["q0"] for b in per]
    tot = [b["d2h"] - b["h2d0"] for b in per]
    # overlap with the previous batch's DSM on ANY stream: did this H2D start
    # before some other batch's DSM ended?
    ends = sorted(b["q1"] for b in per)
    span = (per[-1]["d2h"] - per[0]["h2d0"]) / 1e9
    return {"events": names, "batches": len(per), "streams": len(streams),
            "median_us": {"h2d": us(h2d), "h2d_end_to_front": us(g1), "front": us(fr), "front_end_to_dsm": us(g2),
                          "dsm": us(dsm), "h2d_start_to_d2h_end": us(tot)},
            "p99_us": {"h2d_end_to_front": float(np.percentile(g1, 99)) / 1e3, "front_end_to_dsm": float(np.percentile(g2, 99)) / 1e3,
                       "h2d_start_to_d2h_end": float(np.percentile(tot, 99)) / 1e3},
            "batches_per_s_in_trace": len(per) / span if span > 0 else None}


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--window", type=int, default=6)
    ap.add_argument("--batches", type=int, default=1500)
    ap.add_argument("--analyze", default="")
    a = ap.parse_args()
    if a.analyze:
        print(json.dumps(analyze(a.analyze), indent=1))
    else:
        run(a)
