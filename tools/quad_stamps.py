#!/usr/bin/env python3
"""Cost of a quad-DSM step, lone and under the ring, from a diagnostic
build (-DFD_QUAD_STAMPS, FD_ED25519_LIB=...): every fd_k_dsm_quad wave sums
its main loop's shader cycles (s_memtime) and real time (s_memrealtime,
100 MHz) into device counters, so

  cycles per wave-step   = cycles / steps   (what one wave's step costs)
  effective clock        = cycles / real ticks x 100 MHz (DVFS, per wave)

are read for (a) lone 4,096-signature batches (a batch alone on the
device: 256 waves, one per SIMD on a quarter of the SIMDs) and (b) the C2
ring at 6 and 8 batches in flight (each batch on its 64-CU group beside
the next batch's front end and, past 4 in flight, another batch's DSM).
The PMC passes of tools/pmc_ring.sh give the same kernel's VALU issue
rate without the ring (rocprofv3 serialises dispatches under --pmc).

usage: FD_ED25519_LIB=lib_qstamps.so quad_stamps.py [batches]"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def summary(acc, what):
    w, steps, cyc, rt = (float(x) for x in acc[:4])
    h = acc[8:].astype(np.float64)
    us = (np.arange(256) + 0.5) * 2.0
    cum = np.cumsum(h) / max(h.sum(), 1)
    return {"what": what, "waves": int(w), "steps_per_wave": steps / max(w, 1),
            "cycles_per_wave_step": cyc / max(steps, 1), "effective_clock_ghz": cyc / max(rt, 1) * 0.1,
            "loop_us_mean": rt / max(w, 1) * 0.01, "loop_us_p50": float(us[np.searchsorted(cum, 0.5)]),
            "loop_us_p90": float(us[np.searchsorted(cum, 0.9)])}


def main():
    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
    import torch
    import bench
    import firedancer_amd as fa
    from firedancer_amd import corpus
    L = fa.lib()
    L.fd_ed25519_gpu_quad_acc.argtypes = [ctypes.c_void_p, ctypes.c_int]
    base = corpus.solana_txns(bench.UNIQUE_SIGS, seed=1000, nthreads=16)
    acc = np.zeros(264, np.uint64)

    # (a) lone batches, device-resident (no ring, no neighbour)
    n = bench.BATCH_SIGS
    eng = fa.Engine(0, max_sigs=n, max_blob=1 << 26, depth=1)
    dev = torch.device("cuda", 0)
    sub = corpus.Batch(base.blob, base.desc[:n])
    d_blob = torch.from_numpy(np.concatenate([sub.blob, np.zeros(64, np.uint8)])).to(dev)
    d_desc = torch.from_numpy(sub.desc.view(np.uint8).copy()).to(dev)
    d_out = torch.zeros(n, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    for _ in range(20):
        eng.verify_dev(n, d_blob.data_ptr(), len(sub.blob), d_desc.data_ptr(), d_out.data_ptr(), s)
    torch.cuda.synchronize()
    L.fd_ed25519_gpu_quad_acc(None, 1)
    for _ in range(200):
        eng.verify_dev(n, d_blob.data_ptr(), len(sub.blob), d_desc.data_ptr(), d_out.data_ptr(), s)
        torch.cuda.synchronize()
    L.fd_ed25519_gpu_quad_acc(acc.ctypes.data, 0)
    eng.close()
    print(json.dumps(summary(acc, "lone 4096-signature batches, device-resident, one at a time")), flush=True)

    # (b) the ring, closed loop
    for window in (1, 6, 8):
        L.fd_ed25519_gpu_quad_acc(None, 1)
        r = bench.ring_stream(fa, base, 0, nb, 8, window=window)
        L.fd_ed25519_gpu_quad_acc(acc.ctypes.data, 0)
        out = summary(acc, f"C2 ring, depth 8, {window} in flight")
        out.update(ring_verifies_per_s=r["pcie_inclusive_verifies_per_s"], p99_ms=r["p99_ms"])
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
