"""Per-kernel HIP-event timing of one library build on the C2 workload
(experiments: FD_ED25519_LIB=<variant.so> python tools/time_kernels.py).
Prints prep/decomp/dsm ms averaged over reps; results are not checked.
usage: time_kernels.py [n (default 262144)] [dsm_pool_min (default: the engine's)]"""
import math
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import firedancer_amd as fa
    from firedancer_amd import corpus
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 64 * 4096
    base = corpus.solana_txns(65536, seed=1000, nthreads=16)
    batch = base.tile(int(math.ceil(n / len(base))))
    batch.desc = batch.desc[:n]
    eng = fa.Engine(0, max_sigs=n, max_blob=max(len(batch.blob), 1 << 24))
    if len(sys.argv) > 2:
        eng.dsm_pool_min = int(sys.argv[2])
    dev = torch.device("cuda", 0)
    blob_sz = len(batch.blob)
    d_blob = torch.from_numpy(np.concatenate([batch.blob, np.zeros(64, np.uint8)])).to(dev)
    d_desc = torch.from_numpy(batch.desc.view(np.uint8).copy()).to(dev)
    d_out = torch.zeros(n, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    for _ in range(3):
        eng.verify_dev_timed(n, d_blob.data_ptr(), blob_sz, d_desc.data_ptr(), d_out.data_ptr(), s)
    ks = np.zeros(len(fa.Engine.KERNELS))
    reps = 10
    for _ in range(reps):
        ks += eng.verify_dev_timed(n, d_blob.data_ptr(), blob_sz, d_desc.data_ptr(), d_out.data_ptr(), s)
    ks /= reps
    ok = bool((d_out == 0).all().item())
    print(os.environ.get("FD_ED25519_LIB", "default"), n, "pool_min", eng.dsm_pool_min, " ".join(f"{k[5:]}={v:.4f}" for k, v in zip(fa.Engine.KERNELS, ks)),
          "accepted" if ok else "NOT-ACCEPTED")


if __name__ == "__main__":
    main()
