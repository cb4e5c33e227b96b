#!/usr/bin/env python3
"""Repeated short live-producer runs of the verify tile task (tests/
vt_live.cpp) at one rate, to look at its latency tail: per run the publish
latency percentiles, the shader clock the DSM waves held, and the seq
ranges (~ arrival time at the fixed rate) whose publishes took > --slow-ms.

usage: tools/live_probe.py [--runs 4] [--modes copy,inplace] [--rate 1e6] [--count 34000]"""
import argparse
import json
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def clusters(seqs, gap=64):
    out = []
    for s in seqs:
        if out and s - out[-1][1] <= gap:
            out[-1][1] = s
        else:
            out.append([s, s])
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=4)
    ap.add_argument("--modes", default="copy,inplace")
    ap.add_argument("--rate", type=float, default=1e6, help="frags/s")
    ap.add_argument("--count", type=int, default=34000)
    ap.add_argument("--slow-ms", type=float, default=1.0)
    ap.add_argument("--max-wait-ns", type=int, default=0)
    a = ap.parse_args()
    import firedancer_amd as fa
    from live_common import read_pubout, run, write_frags
    from task_c5 import corpus
    frags = corpus(20000, 77)
    tmp = tempfile.mkdtemp()
    fp, po = os.path.join(tmp, "frags.bin"), os.path.join(tmp, "pub.bin")
    write_frags(fp, frags)
    from live_common import quiet_cpus
    pin = quiet_cpus(2)   # producer k, tile k: the quietest cores of the GPU's NUMA node
    for i in range(a.runs):
        for mode in a.modes.split(","):
            kw = dict(mode=mode, rate=a.rate, count=a.count, depth=16384, batch=4096, eng_depth=8, pubout=po,
                      max_wait_ns=a.max_wait_ns)
            if pin:
                kw["cpus"] = pin
            d = run(os.path.join(ROOT, "firedancer_amd", "vt_live"), fp, timeout=120, **kw)
            pub = read_pubout(po)
            lat = pub[:, 1] / 1e6
            slow = pub[lat > a.slow_ms, 0].astype(np.int64)
            cl = clusters(list(slow))
            print(json.dumps({"run": i, "mode": mode, "rc": d["rc"], "lat": d["lat"], "dsm_ghz": d.get("dsm_ghz"),
                              "dsm_waves": d.get("dsm_waves"), "batches": d["diag"]["BATCH_CNT"],
                              "age_closes": d["diag"]["AGE_CNT"], "slow": len(slow),
                              "tile_ns": d.get("tile_ns"), "tile_max_gap_ms": d.get("tile_max_gap_ms"),
                              "tile_nivcsw": d.get("tile_nivcsw"), "mismatch": d.get("mismatch"),
                              "slow_ranges": [(int(x), int(y), round(float(lat[pub[:, 0] == x][0]), 3)) for x, y in cl[:8]]}),
                  flush=True)


if __name__ == "__main__":
    main()
