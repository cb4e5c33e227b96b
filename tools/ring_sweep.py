#!/usr/bin/env python3
"""C2 ring streaming sweep on one GPU: 4096-signature batches through the
per-GPU feeder (bench.ring_stream) over ring depth x CU groups x window.
One JSON line per configuration.

usage: python3 tools/ring_sweep.py [--batches N] [--depths 3,4,6,8] [--groups 1,2,3,4] [--windows 1,2]
  (window given as a multiple of the depth)"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=4000)
    ap.add_argument("--depths", default="3,4,6,8")
    ap.add_argument("--groups", default="1,2,3,4")
    ap.add_argument("--windows", default="1")
    ap.add_argument("--window-abs", default="", help="comma list of absolute windows (batches in flight), instead of --windows")
    ap.add_argument("--no-register", action="store_true")
    a = ap.parse_args()
    import torch  # noqa: F401  (one HIP runtime, firedancer_amd._share_hip_runtime)
    import bench
    import firedancer_amd as fa
    from firedancer_amd import corpus
    base = corpus.solana_txns(bench.UNIQUE_SIGS, seed=1000, nthreads=min(16, os.cpu_count() or 8))
    for d in [int(x) for x in a.depths.split(",")]:
        for g in [int(x) for x in a.groups.split(",")]:
            if g > d:
                continue
            wins = [int(x) for x in a.window_abs.replace("+", ",").split(",")] if a.window_abs else [int(x) * d for x in a.windows.split(",")]
            for w in wins:
                if w > d:
                    continue
                r = bench.ring_stream(fa, base, 0, a.batches, d, groups=g, window=w, register=not a.no_register)
                print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
