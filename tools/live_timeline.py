#!/usr/bin/env python3
"""Where in time a live-producer run's latency tail sits: runs the verify
tile task harness (tests/vt_live.cpp) with every publish recorded (seq,
tsorig -> tspub), maps each publish to its arrival time (seq / the paced
rate) and prints, per 10 ms window, the windows whose worst publish took
longer than --slow-ms: when they start, how long the slow stretch lasts,
its worst latency, and the gaps between stretches (periodic or random).

usage: tools/live_timeline.py [--mode copy] [--rate 10e6 verifies/s] [--seconds 20]"""
import argparse
import json
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="copy")
    ap.add_argument("--rate", type=float, default=10e6, help="verifies/s")
    ap.add_argument("--seconds", type=float, default=20.0)
    ap.add_argument("--slow-ms", type=float, default=2.0)
    ap.add_argument("--max-wait-ns", type=int, default=0)
    a = ap.parse_args()
    from live_common import quiet_cpus, read_pubout, run, write_frags
    from task_c5 import corpus, fa_sigs
    frags = corpus(20000, 77)
    spf = float(np.mean([fa_sigs(f) for f in frags]))
    tmp = tempfile.mkdtemp()
    fp, po = os.path.join(tmp, "frags.bin"), os.path.join(tmp, "pub.bin")
    write_frags(fp, frags)
    pin = quiet_cpus(2)
    rate = a.rate / spf
    kw = dict(mode=a.mode, rate=rate, seconds=a.seconds, depth=16384, batch=4096, eng_depth=8, pubout=po,
              max_wait_ns=a.max_wait_ns)
    if pin:
        kw["cpus"] = pin
    import resource

    def cg():
        try:
            return dict(line.split() for line in open("/sys/fs/cgroup/cpu.stat"))
        except OSError:
            return {}
    cg0, ru0 = cg(), resource.getrusage(resource.RUSAGE_CHILDREN)
    d = run(os.path.join(ROOT, "firedancer_amd", "vt_live"), fp, timeout=a.seconds + 120, **kw)
    cg1, ru1 = cg(), resource.getrusage(resource.RUSAGE_CHILDREN)
    # the cgroup's CPU quota (cpu.max) throttles every thread of the group
    # once its period's budget is spent: a 100 ms rhythm in the tail
    cgd = {k: int(cg1[k]) - int(cg0.get(k, 0)) for k in ("nr_periods", "nr_throttled", "throttled_usec", "usage_usec")
           if k in cg1}
    try:
        cgd["cpu.max"] = open("/sys/fs/cgroup/cpu.max").read().strip()
    except OSError:
        pass
    harness_cpu_s = (ru1.ru_utime - ru0.ru_utime) + (ru1.ru_stime - ru0.ru_stime)
    pub = read_pubout(po)
    os.unlink(po)
    t_arr = pub[:, 0] / rate                       # s, arrival of each published frag
    lat = pub[:, 1] / 1e6                          # ms
    win = (t_arr / 0.01).astype(np.int64)          # 10 ms windows
    nw = int(win.max()) + 1
    wmax = np.zeros(nw)
    np.maximum.at(wmax, win, lat)
    slow = np.nonzero(wmax > a.slow_ms)[0]
    stretches = []
    for w in slow:
        if stretches and w - stretches[-1][1] <= 1:
            stretches[-1][1] = int(w)
            stretches[-1][2] = max(stretches[-1][2], wmax[w])
        else:
            stretches.append([int(w), int(w), float(wmax[w])])
    starts = np.array([s[0] for s in stretches]) * 0.01
    print(json.dumps({"mode": a.mode, "verifies_s": a.rate, "seconds": a.seconds, "cpus": pin, "lat": d["lat"],
                      "tile_max_gap_ms": d.get("tile_max_gap_ms"), "tile_nivcsw": d.get("tile_nivcsw"),
                      "ring_full": d["diag"]["RING_FULL_CNT"], "batches": d["diag"]["BATCH_CNT"],
                      "cgroup": cgd, "harness_cpus_used": round(harness_cpu_s / d["run_s"], 2),
                      "windows": nw, "slow_windows": int(len(slow)), "stretches": len(stretches),
                      "stretch_ms": [int(10 * (s[1] - s[0] + 1)) for s in stretches[:40]],
                      "stretch_start_s": [round(float(x), 3) for x in starts[:40]],
                      "stretch_worst_ms": [round(s[2], 2) for s in stretches[:40]],
                      "gap_s_median": float(np.median(np.diff(starts))) if len(starts) > 2 else None}), flush=True)


if __name__ == "__main__":
    main()
