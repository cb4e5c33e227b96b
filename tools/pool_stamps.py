#!/usr/bin/env python3
"""Where a fd_k_dsm_pool wave's time goes (diagnostic build with
-DFD_POOL_STAMPS, e.g. make OUT=variants/lib_stamps.so BUILD=build_stamps
EXTRA=-DFD_POOL_STAMPS; run with FD_ED25519_LIB pointing at it): per wave,
s_memtime cycles in selection vs step, by op kind.  The stamps themselves
cost ~10 % of wave time (MI355X_MICROARCH.md)."""
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import firedancer_amd as fa
    from firedancer_amd import corpus
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    base = corpus.solana_txns(65536, seed=1000, nthreads=16)
    b = base.tile((n + len(base) - 1) // len(base))
    eng = fa.Engine(0, max_sigs=n, max_blob=len(base.blob) + 64)
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream(dev).cuda_stream
    d_blob = torch.from_numpy(np.concatenate([base.blob, np.zeros(64, np.uint8)])).to(dev)
    d_desc = torch.from_numpy(b.desc[:n].view(np.uint8).copy()).to(dev)
    d_out = torch.zeros(n, dtype=torch.int32, device=dev)
    for _ in range(2):
        ks = eng.verify_dev_timed(n, d_blob.data_ptr(), len(base.blob), d_desc.data_ptr(), d_out.data_ptr(), s)
    nw = (n + 127) // 128
    buf = np.zeros(nw * 8, np.uint64)
    f = fa.lib().fd_ed25519_gpu_pool_stamps
    f.argtypes = [ctypes.c_void_p, ctypes.c_ulong]
    f.restype = ctypes.c_int
    assert f(buf.ctypes.data, buf.nbytes) == 0
    w = buf.reshape(nw, 8).astype(np.float64)
    tot = w.sum(0)
    out = {"n": n, "waves": nw, "pool_ms": float(ks[3]),
           "per_wave_cycles": float(tot[7] / nw),
           "sel_dbl_frac": float(tot[0] / tot[7]), "step_dbl_frac": float(tot[1] / tot[7]),
           "sel_add_frac": float(tot[3] / tot[7]), "step_add_frac": float(tot[4] / tot[7]),
           "cycles_per_dbl_iter": float(tot[1] / tot[2]), "cycles_per_add_iter": float(tot[4] / tot[5]),
           "sel_cycles_per_iter": float((tot[0] + tot[3]) / (tot[2] + tot[5])),
           "iters_per_wave": float((tot[2] + tot[5]) / nw), "add_iter_frac": float(tot[5] / (tot[2] + tot[5])),
           "lane_occupancy": float(tot[6] / (64 * (tot[2] + tot[5]))),
           "accepted": bool((d_out == 0).all().item())}
    g = getattr(fa.lib(), "fd_ed25519_gpu_pool_stamps2", None)
    if g is not None:
        g.argtypes = [ctypes.c_void_p, ctypes.c_ulong]
        b2 = np.zeros(nw * 4, np.uint64)
        assert g(b2.ctypes.data, b2.nbytes) == 0
        t2 = b2.reshape(nw, 4).astype(np.float64).sum(0)
        it = tot[2] + tot[5]
        out.update(sel_counts_cycles=float(t2[0] / it), sel_walk_cycles=float(t2[1] / it), sel_permute_cycles=float(t2[2] / it))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
