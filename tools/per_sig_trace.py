#!/usr/bin/env python3
"""One thread calling fd_ed25519_verify (the per-signature drop-in) back to
back, for C2-shaped messages (1103/1167 B: 10 SHA-512 blocks) and short
ones (200 B: 3 blocks): per-call latency p50/p99 per message size.  Run it
under `rocprofv3 --kernel-trace` and feed the trace
to `--timeline DIR`: per call, where the time goes (H2D, front end,
DSM, D2H and the gaps between them)."""
import argparse
import csv
import glob
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def calls(n):
    import firedancer_amd as fa
    from firedancer_amd import corpus
    sets = (("c2_1103_1167B", corpus.solana_txns(512, seed=3)), ("short_200B", corpus.simple(512, msg_sz=200, seed=3)))
    fa.verify(sets[0][1].msg(0), sets[0][1].sig(0), sets[0][1].pub(0))        # engine up
    out = {}
    for label, b in sets:
        lat = []
        for i in range(n):
            j = i % len(b)
            t0 = time.perf_counter()
            r = fa.verify(b.msg(j), b.sig(j), b.pub(j))
            lat.append(time.perf_counter() - t0)
            assert r == 0, (label, i, r)
        lat = np.array(lat[10:]) * 1e3
        out[label] = {"calls": len(lat), "p50_ms": float(np.percentile(lat, 50)), "p99_ms": float(np.percentile(lat, 99))}
    return out


def timeline(d):
    """per-call breakdown from a rocprofv3 kernel trace: a call's H2D is a
    blit kernel (__amd_rocclr_copyBuffer) on the slot's stream, then
    fd_k_front and the DSM (fd_k_dsm_oct since round 4; the codes are
    written straight into the slot's pinned memory, so no D2H copy
    follows: a trace from before that shows a second copy, reported as
    d2h_blit_us)"""
    ev = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    ev.sort()
    rows = []
    for i in range(2, len(ev) - 2):
        if "copy" in ev[i-1][2] and "front" in ev[i][2] and "dsm" in ev[i+1][2]:
            c, f, q, o = ev[i-1], ev[i], ev[i+1], ev[i+2]
            nxt = ev[i+3][2] if i + 3 < len(ev) else ""
            d2h = o[1] - o[0] if ("copy" in o[2] and "front" not in nxt) else 0   # o is the next call's H2D when a front follows it
            end = o[1] if d2h else q[1]
            rows.append([c[1] - c[0], f[0] - c[1], f[1] - f[0], max(q[0] - f[1], 0), q[1] - q[0], d2h, end - c[0],
                         c[0] - ev[i-2][1], q[2]])
    if not rows:
        return None
    kern = sorted(set(r[-1] for r in rows))
    a = np.array([r[:-1] for r in rows], dtype=np.float64) / 1e3
    names = ["h2d_blit_us", "h2d_to_front_us", "fd_k_front_us", "front_to_dsm_us", "dsm_us",
             "d2h_blit_us", "device_span_us", "idle_before_call_us"]
    # the calls run in message-size order: the first half C2-shaped, the second short
    h = len(a) // 2
    out = {label: {"calls": len(x), **{n: round(float(np.median(x[:, c])), 1) for c, n in enumerate(names)}}
           for label, x in (("c2_1103_1167B", a[1:h]), ("short_200B", a[h + 1:]))}
    out["dsm_kernels"] = kern
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=300)
    ap.add_argument("--timeline", default="")
    a = ap.parse_args()
    if a.timeline:
        print(json.dumps({"per_call_median_device_timeline": timeline(a.timeline)}))
    else:
        print(json.dumps(calls(a.calls)))
