#!/usr/bin/env python3
"""C5 (BASELINE.json configs[4]) on one GPU: a sustained stream of
QUIC-format frags (Solana-MTU txns, 1..12 signatures, uniform) through
the verify tile (HA dedup -> pinned staging -> GPU batches -> in-order
publish), host-fed from one thread, PCIe included.  Prints one JSON
line: sustained verifies/s and txns/s over --seconds of streaming.

Multi-GPU: run one process per GPU (python -m torch.distributed.run
--nproc-per-node N tools/bench_tile.py); each rank is an independent tile
on its own device and shard, rank 0 prints the sum (replicas, no
collective on the data path)."""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sigs", type=int, default=131072, help="unique signatures in the frag set")
    ap.add_argument("--batch", type=int, default=65536, help="signatures per GPU batch")
    ap.add_argument("--depth", type=int, default=4, help="engine ring slots")
    ap.add_argument("--seconds", type=float, default=10.0)
    a = ap.parse_args()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    import firedancer_amd as fa
    from firedancer_amd import corpus, txn
    from firedancer_amd.tile import VerifyTile

    b = corpus.solana_txns(a.sigs, seed=77 + rank, sig_dist=[1 / 12] * 12, nthreads=16)
    starts = sorted({int(d["sig_off"]) // corpus.TXN_MTU * corpus.TXN_MTU for d in b.desc})
    frags = [txn.frag(bytes(b.blob[s:s + corpus.TXN_MTU])) for s in starts]
    base = np.frombuffer(b"".join(frags), np.uint8).copy()
    sz = np.array([len(f) for f in frags], np.uint32)
    off = np.concatenate([[0], np.cumsum(sz)[:-1]]).astype(np.uint64)

    eng = fa.Engine(local, max_sigs=a.batch, max_blob=a.batch * 1400, depth=a.depth)
    tile = VerifyTile(eng, batch_sigs=a.batch, collect=False)
    tile.rx_burst(base, off, sz)            # warm-up pass
    tile.service(flush=True)
    d0 = tile.diag()
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    passes = 0
    while time.perf_counter() - t0 < a.seconds:
        tile.rx_burst(base, off, sz)
        passes += 1
    tile.service(flush=True)
    el = time.perf_counter() - t0
    d1 = tile.diag()
    sigs = d1["SIG_CNT"] - d0["SIG_CNT"]
    pub = d1["PUB_CNT"] - d0["PUB_CNT"]
    assert d1["SV_FILT_CNT"] == 0 and pub == passes * len(frags)
    tot = np.array([sigs, pub, el])
    if dist:
        t = torch.tensor(tot, dtype=torch.float64, device="cuda")
        dist.all_reduce(t[:2])
        m = t[2:].clone()
        dist.all_reduce(m, op=dist.ReduceOp.MAX)
        tot = np.array([t[0].item(), t[1].item(), m.item()])
    if rank == 0:
        print(json.dumps({"metric": "sustained verify-tile stream (C5)", "value": tot[0] / tot[2],
                          "unit": "verifies/s", "txns_per_s": tot[1] / tot[2], "n_gpus": world,
                          "seconds": tot[2], "batch_sigs": a.batch, "depth": a.depth,
                          "frags_per_pass": len(frags), "sigs_per_pass": a.sigs,
                          "sig_dist": "uniform 1..12 per txn, 1232-byte txns", "pcie_inclusive": True,
                          "diag": d1}), flush=True)
    tile.close()
    eng.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
