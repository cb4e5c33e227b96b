#!/usr/bin/env python3
"""The C2 ring's closed-loop (6 and 8 in flight) and open-loop (offered
34 / 36 / 38 M verifies/s) points alone, on the bench's C3-mix ring corpus
with every code checked against the reference build (bench.ring_stream):
one JSON line.  For same-box A/B of library variants (FD_ED25519_LIB).
usage: ring_paced.py [batches (default 4000)] [offered M/s, ... (default 34,36,38)]
FD_RING_DEPTH (default 8): the ring depth (open loop: up to 2 x depth outstanding);
the line records it and GPU_MAX_HW_QUEUES."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 4000
    loads = [float(x) for x in sys.argv[2:]] or [34, 36, 38]
    import torch  # noqa: F401  (one HIP runtime)
    import bench
    import firedancer_amd as fa
    from firedancer_amd import corpus
    ring = corpus.c3_windows(bench.RING_WINDOWS, bench.BATCH_SIGS, seed=4242, extra=[
        (bytes.fromhex(m), bytes.fromhex(s), bytes.fromhex(p)) for m, s, p in corpus.Q2_VECTORS],
        extra_at=bench.RING_Q2_AT, nthreads=min(16, os.cpu_count() or 8))
    exp = bench.ring_reference_codes(ring, bench.usable_cores())
    depth = int(os.environ.get("FD_RING_DEPTH", "8"))
    out = {"depth": depth, "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES")}
    for w in sorted({6, 8, depth}):
        r = bench.ring_stream(fa, ring, 0, nb, depth, window=w, expected=exp)
        out[f"closed_w{w}"] = {"mps": r["pcie_inclusive_verifies_per_s"] / 1e6, "p50_ms": r["p50_ms"], "p99_ms": r["p99_ms"],
                               "mismatches": r["mismatches"]}
    for mps in loads:
        r = bench.ring_stream(fa, ring, 0, nb, depth, window=2 * depth, period_ns=int(round(bench.BATCH_SIGS / (mps * 1e6) * 1e9)), expected=exp)
        out[f"paced_{mps:g}"] = {"mps": r["pcie_inclusive_verifies_per_s"] / 1e6, "sched_p50_ms": r["sched_to_done_p50_ms"],
                                 "sched_p99_ms": r["sched_to_done_p99_ms"], "sched_max_ms": r["sched_to_done_max_ms"],
                                 "push_submit_p99_ms": r["push_to_submit_p99_ms"], "submit_done_p99_ms": r["submit_to_done_p99_ms"],
                                 "mismatches": r["mismatches"]}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
