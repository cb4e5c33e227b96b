#!/usr/bin/env python3
"""Driver for PMC passes over the latency schedule's kernels (fd_k_front,
fd_k_dsm_quad; round 4 also ran the since-removed two-waves-per-SIMD
fd_k_dsm_quad2, profiles/r04_pmc_ring.json): device-resident C2 batches of n signatures
verified one at a time on a depth-1 engine (the whole device), so each
dispatch's counters are its own (rocprofv3 --pmc serialises dispatches).

  n = 4096   one batch: 256 quad waves, one per SIMD on a quarter of them
  n = 16384  1,024 waves: one per SIMD on every SIMD
  n = 32768  2,048 waves: the quad (34.6 KiB of LDS) runs them in two
             rounds of one per SIMD
  oct n <= 64: the per-signature drop-in's eight-lane DSM (fd_k_dsm_oct),
             n / 8 waves

usage: pmc_ring.py quad|oct <n> [reps]"""
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    sched, n = sys.argv[1], int(sys.argv[2])
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    import torch
    import firedancer_amd as fa
    from firedancer_amd import corpus
    base = corpus.solana_txns(65536, seed=1000, nthreads=16)
    b = base.tile(int(math.ceil(n / len(base))))
    b.desc = b.desc[:n]
    eng = fa.Engine(0, max_sigs=n, max_blob=max(len(b.blob), 1 << 24), depth=1)
    eng.dsm_quad_max = max(eng.dsm_quad_max, n)
    if sched == "oct":
        if n > eng.dsm_oct_max:
            raise SystemExit("the eight-lane DSM takes batches of at most dsm_oct_max")
    elif sched != "quad":
        raise SystemExit("schedules: quad, oct (round 4)")
    dev = torch.device("cuda", 0)
    d_blob = torch.from_numpy(np.concatenate([b.blob, np.zeros(64, np.uint8)])).to(dev)
    d_desc = torch.from_numpy(b.desc.view(np.uint8).copy()).to(dev)
    d_out = torch.zeros(n, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    for _ in range(reps):
        eng.verify_dev(n, d_blob.data_ptr(), len(b.blob), d_desc.data_ptr(), d_out.data_ptr(), s)
        torch.cuda.synchronize()
    ok = bool((d_out == 0).sum().item() >= n - 4)
    print(sched, n, reps, "accepted" if ok else "NOT-ACCEPTED", flush=True)
    eng.close()


if __name__ == "__main__":
    main()
