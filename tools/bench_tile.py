#!/usr/bin/env python3
"""C5 (BASELINE.json configs[4]): a sustained stream of QUIC-format frags
(Solana-MTU txns, 1..12 signatures, uniform) through verify tiles (HA
dedup -> pinned staging -> GPU batches -> in-order publish), each tile
host-fed from its own thread pinned to its GPU's NUMA node, PCIe
included.  Prints one JSON line: sustained verifies/s and txns/s over
--seconds of streaming.

--latency: each frag's tsorig is its receipt time and the publish
callback (native) histograms tsorig -> tspub; --curve 4096,16384,...
prints one such point per batch size.  --multi: ONE tile in the
multi-engine feeder mode over all the engines (fd_verify_tile_new_multi).

--check-window W: before the timed stream, the first W frags of the set go
through a collecting tile of the same layout (engines, mode, batch size)
and the line records what it published (the ordered ctl = frag indices,
as a sha256 and a count) and its counters; tests/test_c5_record.py holds
that record against the reference's per-frag semantics
(fd_frank_verify_synth_load.c:360-410: its tcache and fd_ed25519_verify)
on the same frags, regenerated from the seed.

Multi-GPU, one process: --gpus N runs --tiles tiles on each of devices
0..N-1 (tile k on device k mod N), every tile an independent replica on
its own engine, ring and frag stream (no collective on the data path).
Multi-GPU, one process per GPU: python -m torch.distributed.run
--nproc-per-node N tools/bench_tile.py; rank 0 prints the sum.
FD_BENCH_SHARE_GPU=1 lets --gpus exceed the visible devices (rehearsal
on one GPU)."""
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
    ap.add_argument("--tiles", type=int, default=1, help="verify tiles per GPU (one host thread + engine each)")
    ap.add_argument("--gpus", type=int, default=1, help="devices driven from this process, one tile set each")
    ap.add_argument("--multi", action="store_true",
                    help="one tile in the multi-engine feeder mode driving --tiles engines on each of --gpus devices")
    ap.add_argument("--inplace", action="store_true",
                    help="in-place tiles (fd_verify_tile_new_inplace): frags DMA'd from the frag set itself, no copy")
    ap.add_argument("--latency", action="store_true",
                    help="stamp tsorig at each frag's receipt and report tsorig -> tspub percentiles (native histogram)")
    ap.add_argument("--curve", default="", help="comma-separated batch sizes: one latency point per size (implies --latency)")
    ap.add_argument("--check-window", type=int, default=0,
                    help="record the publish stream of the first W frags (tests/test_c5_record.py checks it)")
    a = ap.parse_args()
    if a.curve:
        a.latency = True
        for bs in [int(x) for x in a.curve.split(",")]:
            a.batch = bs
            run(a)
        return
    run(a)


def run(a):
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    dist = None
    share = os.environ.get("FD_BENCH_SHARE_GPU") == "1"     # rehearsal: ranks share the visible GPUs
    if share:
        local = local % max(1, torch.cuda.device_count())
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        if share:
            dist.init_process_group("gloo")
        else:
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

    import threading
    ndev = fa.device_count()
    if a.gpus > ndev and os.environ.get("FD_BENCH_SHARE_GPU") != "1":
        raise SystemExit(f"--gpus {a.gpus} but {ndev} gfx950 devices visible")
    devs = [local if world > 1 else (k % a.gpus) % max(ndev, 1) for k in range(a.tiles * a.gpus)]
    engs = [fa.Engine(d, max_sigs=a.batch, max_blob=a.batch * 1400, depth=a.depth) for d in devs]
    from firedancer_amd.tile import LatHist
    check = None
    if a.check_window:
        # the sample window: a collecting tile of the same layout over the
        # first W frags (fresh tcache), published ctl (= frag index) in order
        # (with corpus.c5_check_edits: rejected signatures, dedup hits and
        # frags that do not parse among them)
        W = min(a.check_window, len(frags))
        cf = corpus.c5_check_edits(frags[:W])
        cbase = np.frombuffer(b"".join(cf), np.uint8).copy()
        csz = np.array([len(f) for f in cf], np.uint32)
        coff = np.concatenate([[0], np.cumsum(csz)[:-1]]).astype(np.uint64)
        ct = VerifyTile(engs if a.multi else engs[0], batch_sigs=a.batch, collect=True,
                        region=cbase if a.inplace else None)
        ct.rx_burst(cbase, coff, csz, ctl=np.arange(W, dtype=np.uint64))
        ct.service(flush=True)
        pub_ctl = np.array([p[2] for p in ct.published], np.uint64)
        import hashlib
        check = {"frags": W, "published": int(len(pub_ctl)), "pub_ctl_sha256": hashlib.sha256(pub_ctl.tobytes()).hexdigest(),
                 "diag": {k: int(v) for k, v in ct.diag().items()}, "seed": 77 + rank, "sigs": a.sigs,
                 "edits": "corpus.c5_check_edits"}
        ct.close()
    if a.multi:       # one tile, every engine behind its feeder
        lats = [LatHist()] if a.latency else [None]
        tiles = [VerifyTile(engs, batch_sigs=a.batch, collect=False, lat=lats[0], region=base if a.inplace else None)]
        devs = devs[:1]
    else:
        lats = [LatHist() if a.latency else None for _ in engs]
        tiles = [VerifyTile(e, batch_sigs=a.batch, collect=False, lat=h, region=base if a.inplace else None)
                 for e, h in zip(engs, lats)]
    for tile in tiles:
        tile.rx_burst(base, off, sz)            # warm-up pass
        tile.service(flush=True)
    for h in lats:
        if h is not None:
            h.reset()
    d0s = [tile.diag() for tile in tiles]
    if dist:
        dist.barrier()
    passes = [0] * len(tiles)
    cpus = {d: fa.numa_cpus(d) for d in set(devs)}
    t0 = time.perf_counter()

    def feed(k):
        # the feeding thread on its GPU's NUMA node
        if cpus[devs[k]]:
            os.sched_setaffinity(0, cpus[devs[k]])
        # ctypes drops the GIL inside rx_burst: the tiles' host feeds run in parallel
        while time.perf_counter() - t0 < a.seconds:
            if a.latency:
                tiles[k].rx_burst_now(base, off, sz)
            else:
                tiles[k].rx_burst(base, off, sz)
            passes[k] += 1
        tiles[k].service(flush=True)
    th = [threading.Thread(target=feed, args=(k,)) for k in range(len(tiles))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    el = time.perf_counter() - t0
    sigs = pub = 0
    for d0, tile, p in zip(d0s, tiles, passes):
        d1 = tile.diag()
        sigs += d1["SIG_CNT"] - d0["SIG_CNT"]
        pb = d1["PUB_CNT"] - d0["PUB_CNT"]
        pub += pb
        # every pass carries the same frags: the same txns fail verification each
        # pass (the reference's own rejects, e.g. Q2 limb-alias cases: seed 77 x
        # 524288 signatures holds one, index 171140, ERR_MSG in the reference)
        svf = d1["SV_FILT_CNT"] - d0["SV_FILT_CNT"]
        assert svf == p * d0["SV_FILT_CNT"] and pb + svf == p * len(frags), (d0, d1, p, len(frags))
    d0 = d0s[0]
    tot = np.array([sigs, pub, el])
    if dist:
        t = torch.tensor(tot, dtype=torch.float64, device="cpu" if share else "cuda")
        dist.all_reduce(t[:2])
        m = t[2:].clone()
        dist.all_reduce(m, op=dist.ReduceOp.MAX)
        tot = np.array([t[0].item(), t[1].item(), m.item()])
    if rank == 0:
        print(json.dumps({"metric": "sustained verify-tile stream (C5)", "value": tot[0] / tot[2],
                          "unit": "verifies/s", "txns_per_s": tot[1] / tot[2],
                          "n_gpus": world if world > 1 else a.gpus, "devices": sorted(set(devs)),
                          "numa_nodes": {d: fa.lib().fd_ed25519_gpu_device_numa_node(d) for d in sorted(set(devs))},
                          "seconds": tot[2], "batch_sigs": a.batch, "depth": a.depth, "tiles_per_gpu": a.tiles,
                          "frags_per_pass": len(frags), "sigs_per_pass": a.sigs,
                          "sig_dist": "uniform 1..12 per txn, 1232-byte txns", "pcie_inclusive": True,
                          "sv_filt_per_pass": int(d0["SV_FILT_CNT"]),
                          "multi_engine_tile": bool(a.multi), "inplace": bool(a.inplace), "engines": len(engs),
                          "latency_tsorig_to_tspub": lat_summary(lats) if a.latency else None,
                          "check_window": check,
                          "diag": d1}), flush=True)
    for tile in tiles:
        tile.close()
    for e in engs:
        e.close()
    if dist:
        dist.destroy_process_group()


def lat_summary(lats):
    """merge the tiles' histograms: tsorig (frag received) -> tspub
    (published after its batch's codes reached the host), PCIe included"""
    from firedancer_amd.tile import LatHist
    m = LatHist()
    for h in lats:
        m.buf[0] += h.buf[0]
        m.buf[1] += h.buf[1]
        m.buf[2] = max(m.buf[2], h.buf[2])
        m.buf[3] += h.buf[3]
        m.buf[4:] += h.buf[4:]
    return m.summary()


if __name__ == "__main__":
    main()
