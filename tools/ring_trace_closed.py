#!/usr/bin/env python3
"""A closed-loop C2 ring run for a kernel trace: `window` 4,096-signature
batches outstanding on the depth-8 ring (bench.ring_stream, C3-mix
corpus) for `batches` batches.  Run under rocprofv3 --kernel-trace
--memory-copy-trace and read with tools/ring_trace_stats.py.
usage: ring_trace_closed.py [batches (2000)] [window (8)]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    w = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    import torch  # noqa: F401
    import bench
    import firedancer_amd as fa
    from firedancer_amd import corpus
    ring = corpus.c3_windows(bench.RING_WINDOWS, bench.BATCH_SIGS, seed=4242, nthreads=min(16, os.cpu_count() or 8))
    r = bench.ring_stream(fa, ring, 0, nb, 8, window=w, expected=None)
    print(json.dumps({"batches": nb, "window": w, "mps": r["pcie_inclusive_verifies_per_s"] / 1e6,
                      "p50_ms": r["p50_ms"], "p99_ms": r["p99_ms"]}), flush=True)


if __name__ == "__main__":
    main()
