#!/usr/bin/env python3
"""fd_k_dsm_pool time per signature vs launch size (waves in rounds of
2 per SIMD): separates the steady-state rate from the launch tail.
python3 tools/pool_rounds.py [n ...]"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import firedancer_amd as fa
    from firedancer_amd import corpus
    sizes = [int(x) for x in sys.argv[1:]] or [262144, 524288, 1048576, 2097152]
    base = corpus.solana_txns(65536, seed=1000, nthreads=16)
    eng = fa.Engine(0, max_sigs=max(sizes), max_blob=len(base.blob) + 64)
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream(dev).cuda_stream
    d_blob = torch.from_numpy(np.concatenate([base.blob, np.zeros(64, np.uint8)])).to(dev)
    for n in sizes:
        b = base.tile((n + len(base) - 1) // len(base))
        d_desc = torch.from_numpy(b.desc[:n].view(np.uint8).copy()).to(dev)
        d_out = torch.zeros(n, dtype=torch.int32, device=dev)
        for _ in range(2):
            eng.verify_dev_timed(n, d_blob.data_ptr(), len(base.blob), d_desc.data_ptr(), d_out.data_ptr(), s)
        ks = np.mean([eng.verify_dev_timed(n, d_blob.data_ptr(), len(base.blob), d_desc.data_ptr(), d_out.data_ptr(), s)
                      for _ in range(5)], axis=0)
        ok = bool((d_out == 0).all().item())
        print(json.dumps({"lib": os.environ.get("FD_ED25519_LIB", "default"), "n": n, "waves": n // 128,
                          "pool_ms": float(ks[3]), "pool_ns_per_sig": float(ks[3]) * 1e6 / n,
                          "total_ms": float(ks.sum()), "accepted": ok}), flush=True)


if __name__ == "__main__":
    main()
