#!/usr/bin/env python3
"""Per-wave front-end times of LONE 4096-signature C2 launches (one batch
on the whole device, no ring): a diagnostic build (-DFD_FRONT_STAMPS,
FD_ED25519_LIB=...) histograms each fd_k_front wave's duration -- prep
round waves, prep schedule waves (two-wave SHA-512) and decomp waves --
beside the launch's HIP-event front-end time.
Round 4: per-signature stamps of the round wave's tail (sc_reduce, op-row
zeroing + recoder; these are per active lane), and any batch size n.
usage: FD_ED25519_LIB=lib_stamps.so front_lone.py [launches] [n]"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    import torch
    import firedancer_amd as fa
    from firedancer_amd import corpus
    L = fa.lib()
    L.fd_ed25519_gpu_front_hist.argtypes = [ctypes.c_void_p, ctypes.c_int]
    base = corpus.solana_txns(65536, seed=1000, nthreads=16)
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    d = base.desc[:n].copy()
    hi = int(max((d["msg_off"] + d["msg_sz"]).max(), d["sig_off"].max() + 64))
    blob = np.ascontiguousarray(base.blob[:hi])
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream(dev).cuda_stream
    d_blob = torch.from_numpy(np.concatenate([blob, np.zeros(64, np.uint8)])).to(dev)
    d_desc = torch.from_numpy(d.view(np.uint8).copy()).to(dev)
    d_out = torch.zeros(n, dtype=torch.int32, device=dev)
    eng = fa.Engine(0, max_sigs=1 << 14, max_blob=1 << 26, depth=1)
    for _ in range(5):
        eng.verify_dev_timed(n, d_blob.data_ptr(), len(blob), d_desc.data_ptr(), d_out.data_ptr(), s)
    L.fd_ed25519_gpu_front_hist(None, 1)
    ks = np.array([eng.verify_dev_timed(n, d_blob.data_ptr(), len(blob), d_desc.data_ptr(), d_out.data_ptr(), s)
                   for _ in range(reps)])
    h = np.zeros((6, 256), np.uint64)   # fd_front_hist[6][256]
    L.fd_ed25519_gpu_front_hist(h.ctypes.data, 0)
    out = {"lib": os.environ.get("FD_ED25519_LIB", "default"), "front_ms": float(np.median(ks[:, 0])),
           "accepted": int((d_out == 0).sum().item())}
    out["n"] = n
    for k, name in enumerate(("prep_rounds", "decomp", "prep_schedule", "prep_rounds_to_digest", "sc_reduce", "row_and_recode")):
        c = h[k].astype(np.float64)
        us = (np.arange(256) + 0.5) * (2.0 if k < 4 else 0.2)
        tot = c.sum()
        if not tot:
            continue
        cum = np.cumsum(c) / tot
        out[name] = {"waves": int(tot), "mean_us": float((c * us).sum() / tot),
                     "p50_us": float(us[np.searchsorted(cum, 0.5)]), "p90_us": float(us[np.searchsorted(cum, 0.9)]),
                     "max_us": float(us[np.nonzero(c)[0].max()])}
    print(json.dumps(out), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
