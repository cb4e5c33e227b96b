#!/usr/bin/env python3
"""Where the C2 ring's latency tail comes from: 4096-signature batches
through the feeder (as bench.ring_stream), every job's push / submit /
done host timestamps kept; prints the p50/p99 of push->submit (waiting
for a slot or for the feeder thread) and submit->done (device + queueing
on a CU group + the feeder noticing completion), and for the slowest 1 %
of batches how many other batches completed during their submit->done
window and the largest gap between consecutive completions around them
(a host stall freezes every slot at once; a device-side delay does not).
usage: ring_tail.py [--batches N] [--depth 8] [--window 6] [--groups 4]"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=6000)
    ap.add_argument("--depth", type=int, default=8)
    ap.add_argument("--window", type=int, default=6)
    ap.add_argument("--groups", type=int, default=0)
    ap.add_argument("--gc-off", type=int, default=1, help="1: no garbage-collector pauses in the producer loop")
    a = ap.parse_args()
    import torch  # noqa: F401
    import bench
    import firedancer_amd as fa
    from firedancer_amd import corpus
    base = corpus.solana_txns(bench.UNIQUE_SIGS, seed=1000, nthreads=min(16, os.cpu_count() or 8))
    eng = fa.Engine(0, max_sigs=bench.BATCH_SIGS, max_blob=8 << 20, depth=a.depth)
    if a.groups:
        eng.cu_groups = a.groups
    eng.register(base.blob)
    feeder = fa.Feeder(eng)
    B = bench.BATCH_SIGS
    starts = np.random.default_rng(7).integers(0, len(base) - B, 64)
    descs = [np.ascontiguousarray(base.desc[s:s + B]) for s in starts]
    W = a.window
    jobs = [fa.Job() for _ in range(W)]
    outs = [np.full(B, 99, np.int32) for _ in range(W)]
    rec = []

    def done(k):
        feeder.wait(jobs[k])
        j = jobs[k]
        rec.append((j.t_push_ns, j.t_submit_ns, j.t_done_ns))

    import gc
    if a.gc_off:
        gc.disable()
    for i in range(a.batches):
        k = i % W
        if i >= W:
            done(k)
        feeder.push(base.blob, descs[i % len(descs)], outs[k], jobs[k])
    for i in range(a.batches, a.batches + W):
        if i >= W:
            done(i % W)
    gc.enable()
    feeder.close()
    groups = eng.cu_groups
    eng.close()
    r = np.array(rec[W:], dtype=np.float64) * 1e-6        # ms
    push, sub, dn = r[:, 0], r[:, 1], r[:, 2]
    lat, wait, dev = dn - push, sub - push, dn - sub
    comp = np.sort(dn)
    gaps = np.diff(comp)
    thr = np.percentile(lat, 99)
    slow = np.nonzero(lat >= thr)[0]
    info = []
    for i in slow[:40]:
        inside = int(((comp > sub[i]) & (comp < dn[i])).sum())
        lo, hi = np.searchsorted(comp, sub[i]), np.searchsorted(comp, dn[i])
        g = float(gaps[max(lo - 1, 0):max(hi, lo)].max()) if hi > lo else 0.0
        info.append({"lat": round(float(lat[i]), 3), "wait": round(float(wait[i]), 3), "dev": round(float(dev[i]), 3),
                     "completions_inside": inside, "max_completion_gap": round(g, 3), "t": round(float(push[i] - push[0]), 1)})
    print(json.dumps({"batches": len(r), "depth": a.depth, "window": W, "groups": groups, "gc_off": a.gc_off,
                      "lat_p50": float(np.percentile(lat, 50)), "lat_p99": float(thr),
                      "wait_p50": float(np.percentile(wait, 50)), "wait_p99": float(np.percentile(wait, 99)),
                      "dev_p50": float(np.percentile(dev, 50)), "dev_p99": float(np.percentile(dev, 99)),
                      "completion_gap_p50": float(np.percentile(gaps, 50)), "completion_gap_p99": float(np.percentile(gaps, 99)),
                      "completion_gap_max": float(gaps.max()), "slowest": info}))


if __name__ == "__main__":
    main()
