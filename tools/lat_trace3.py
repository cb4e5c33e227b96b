"""Depth-3 ring latency under a kernel + memory-copy trace: 300 single
4096-signature C2 batches through the engine's pinned ring (bench.py's
latency loop), for the per-stream overlap analysis.
rocprofv3 --kernel-trace --memory-copy-trace -- python3 tools/lat_trace3.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch  # noqa: F401  (HIP runtime before the engine, as bench.py)
    import bench
    import firedancer_amd as fa
    from firedancer_amd import corpus
    base = corpus.solana_txns(65536, seed=1000, nthreads=16)
    eng = fa.Engine(0, max_sigs=1 << 16, max_blob=1 << 24)
    bench.latency(eng, base, 50)
    print(json.dumps(bench.latency(eng, base, 300)), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
