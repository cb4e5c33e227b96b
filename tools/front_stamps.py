#!/usr/bin/env python3
"""Per-wave execution time of the latency front end (fd_k_front) on the
C2 ring, from a diagnostic build (-DFD_FRONT_STAMPS, FD_ED25519_LIB=...):
histograms of prep and decomp wave durations over every batch of a
tools/ring_sweep.py-style stream at the given ring depth / window.
Distinguishes waves that run slowly from waves that start late.
usage: FD_ED25519_LIB=lib_stamps.so front_stamps.py <depth> <window> [batches] [group_always]"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    depth, window = int(sys.argv[1]), int(sys.argv[2])
    nb = int(sys.argv[3]) if len(sys.argv) > 3 else 2000
    import torch  # noqa: F401
    import bench
    import firedancer_amd as fa
    from firedancer_amd import corpus
    L = fa.lib()
    L.fd_ed25519_gpu_front_hist.argtypes = [ctypes.c_void_p, ctypes.c_int]
    base = corpus.solana_txns(bench.UNIQUE_SIGS, seed=1000, nthreads=16)
    h = np.zeros((6, 256), np.uint64)   # fd_front_hist[6][256]
    L.fd_ed25519_gpu_front_hist(None, 1)
    r = bench.ring_stream(fa, base, 0, nb, depth, groups=min(depth, 4), window=window)
    L.fd_ed25519_gpu_front_hist(h.ctypes.data, 0)
    out = {"depth": depth, "window": window, "p50_ms": r["p50_ms"], "p99_ms": r["p99_ms"],
           "group_always": os.environ.get("FD_ED25519_GPU_GROUP_ALWAYS", "0")}
    for k, name in enumerate(("prep", "decomp", "prep_schedule_wave", "prep_round_wave_to_digest")):
        c = h[k].astype(np.float64)
        us = (np.arange(256) + 0.5) * 2.0
        tot = c.sum()
        cum = np.cumsum(c) / max(tot, 1)
        out[name] = {"waves": int(tot), "mean_us": float((c * us).sum() / max(tot, 1)),
                     "p50_us": float(us[np.searchsorted(cum, 0.5)]), "p90_us": float(us[np.searchsorted(cum, 0.9)])}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
