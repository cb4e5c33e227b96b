#!/usr/bin/env python3
"""Per-batch timeline of the C2 ring from a rocprofv3 kernel + memory-copy
trace (tools/ring_trace_closed.py under rocprofv3): for each fd_k_dsm_quad
dispatch, its duration, the gap since the previous quad DSM finished on
the same stream, and the fd_k_front of the same stream before it (its
duration and how long the DSM waited after it).  A group's period is then
split into loop, waiting for its own front end, and idle.
usage: ring_trace_stats.py <kernel_trace.csv> [memory_copy_trace.csv]"""
import csv
import json
import sys

import numpy as np


def pct(x, q):
    return float(np.percentile(np.asarray(x, float), q)) if len(x) else None


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    ev = []
    for r in rows:
        name = r["Kernel_Name"]
        if name.startswith("fd_k_front") or name.startswith("fd_k_dsm_quad"):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name[:14], r.get("Stream_Id") or r.get("Queue_Id")))
    ev.sort()
    t0 = ev[0][0]
    quads = [e for e in ev if e[2].startswith("fd_k_dsm_quad")]
    fronts = [e for e in ev if e[2].startswith("fd_k_front")]
    qd = [(e[1] - e[0]) * 1e-3 for e in quads]
    fd = [(e[1] - e[0]) * 1e-3 for e in fronts]
    # the front end of the same stream that ended last before each quad started
    wait, gapq = [], []
    last_front = {}
    last_quad_end = {}
    for s, e, n, st in ev:
        if n.startswith("fd_k_front"):
            last_front[st] = (s, e)
        else:
            f = last_front.get(st)
            if f:
                wait.append((s - f[1]) * 1e-3)
    # all quads in start order: overlap structure
    ends = sorted(e[1] for e in quads)
    span = (quads[-1][1] - quads[0][0]) * 1e-3
    out = {"quad_dsm_us": {"n": len(qd), "p50": pct(qd, 50), "p90": pct(qd, 90), "p99": pct(qd, 99)},
           "front_us": {"n": len(fd), "p50": pct(fd, 50), "p90": pct(fd, 90), "p99": pct(fd, 99)},
           "front_end_to_quad_start_us": {"p10": pct(wait, 10), "p50": pct(wait, 50), "p90": pct(wait, 90)},
           "quads_per_ms": len(quads) / max(span * 1e-3, 1e-9) * 1e-3,
           "span_ms": span * 1e-3}
    # concurrency of quad DSMs over time (how many run at once)
    pts = sorted([(e[0], 1) for e in quads] + [(e[1], -1) for e in quads])
    cur, last, acc = 0, pts[0][0], {}
    for t, d in pts:
        acc[cur] = acc.get(cur, 0) + (t - last)
        cur += d
        last = t
    tot = sum(acc.values())
    out["quad_concurrency_time_frac"] = {str(k): round(v / tot, 4) for k, v in sorted(acc.items())}
    pts = sorted([(e[0], 1) for e in fronts] + [(e[1], -1) for e in fronts])
    cur, last, acc = 0, pts[0][0], {}
    for t, d in pts:
        acc[cur] = acc.get(cur, 0) + (t - last)
        cur += d
        last = t
    tot = sum(acc.values())
    out["front_concurrency_time_frac"] = {str(k): round(v / tot, 4) for k, v in sorted(acc.items())}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
