"""Small-batch latency breakdown: per-kernel HIP-event ms for one launch
of n signatures (C2 corpus, HBM-resident), and submit->poll wall latency
of single batches through the pinned ring at depth 1 and depth 3.
python tools/latency_breakdown.py [n ...]"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import firedancer_amd as fa
    from firedancer_amd import corpus
    sizes = [int(x) for x in sys.argv[1:]] or [1024, 4096, 16384]
    quad = os.environ.get("FD_QUAD_MAX")
    base = corpus.solana_txns(65536, seed=1000, nthreads=16)
    dev = torch.device("cuda", 0)
    eng = fa.Engine(0, max_sigs=1 << 18, max_blob=1 << 29, depth=3)
    if quad is not None:
        eng.dsm_quad_max = int(quad)
    s = torch.cuda.current_stream(dev).cuda_stream
    pool = os.environ.get("FD_POOL_MIN")
    if pool is not None:
        eng.dsm_pool_min = int(pool)
    for n in sizes:
        src = base if n <= len(base) else base.tile((n + len(base) - 1) // len(base))
        d = src.desc[:n].copy()
        hi = int(max((d["msg_off"] + d["msg_sz"]).max(), d["sig_off"].max() + 64))
        blob = np.ascontiguousarray(src.blob[:hi])
        blob_sz = len(blob)
        d_blob = torch.from_numpy(np.concatenate([blob, np.zeros(64, np.uint8)])).to(dev)
        d_desc = torch.from_numpy(d.view(np.uint8).copy()).to(dev)
        d_out = torch.zeros(n, dtype=torch.int32, device=dev)
        for _ in range(5):
            eng.verify_dev_timed(n, d_blob.data_ptr(), blob_sz, d_desc.data_ptr(), d_out.data_ptr(), s)
        reps = 30
        ks = np.zeros((reps, len(fa.Engine.KERNELS)))
        for r in range(reps):
            ks[r] = eng.verify_dev_timed(n, d_blob.data_ptr(), blob_sz, d_desc.data_ptr(), d_out.data_ptr(), s)
        ok = bool((d_out == 0).all().item())
        # device-resident wall per launch (no events)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(reps):
            eng.verify_dev(n, d_blob.data_ptr(), blob_sz, d_desc.data_ptr(), d_out.data_ptr(), s)
        torch.cuda.synchronize()
        dev_ms = (time.perf_counter() - t) / reps * 1e3
        # depth-1 host round trip
        out = np.zeros(n, np.int32)
        lat = []
        for _ in range(40):
            ts = time.perf_counter()
            tk = eng.submit(blob, d)
            eng.poll(tk, out, block=True)
            lat.append((time.perf_counter() - ts) * 1e3)
        lat = np.array(lat[5:])
        print(json.dumps({"n": n, "quad_max": eng.dsm_quad_max, "pool_min": eng.dsm_pool_min, "accepted": ok,
                          "kernel_ms_mean": {k: float(v) for k, v in zip(fa.Engine.KERNELS, ks.mean(0))},
                          "kernel_sum_ms": float(ks.sum(1).mean()),
                          "dev_launch_ms": dev_ms,
                          "depth1_p50_ms": float(np.percentile(lat, 50)),
                          "depth1_p99_ms": float(np.percentile(lat, 99))}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
