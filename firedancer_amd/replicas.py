"""Multi-GPU plumbing for the replica layout.

Signatures are independent: N processes (one per GPU, launched by
torch.distributed.run) each verify their own shard; nothing is reduced
on the data path.  torch.distributed (RCCL on GPUs, gloo in CPU tests)
carries only the timing barrier, the max-over-ranks of the timed region
and, when a caller wants one, the host-side gather of the per-shard
accept bitmaps.  bench.py and tools/bench_tile.py use these helpers;
tests/test_replicas.py runs them with gloo at world size 2.
"""
from __future__ import annotations

import time

import numpy as np


def shard(total: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous [lo, hi) share of `total` units for `rank`."""
    return total * rank // world, total * (rank + 1) // world


def timed_steps(step, steps: int, dist=None, sync=None, device="cpu") -> float:
    """Run step() `steps` times bracketed by barrier + sync on both sides;
    returns the wall time, max over ranks."""
    if dist is not None:
        dist.barrier()
    if sync:
        sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    if sync:
        sync()
    if dist is not None:
        dist.barrier()
    el = time.perf_counter() - t0
    if dist is not None:
        import torch
        t = torch.tensor([el], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    return el


def all_true(flag: bool, dist=None, device="cpu") -> bool:
    if dist is None:
        return bool(flag)
    import torch
    t = torch.tensor([1 if flag else 0], dtype=torch.int32, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t.item())


def gather_bitmap(codes: np.ndarray, total: int, dist=None, device="cpu"):
    """Host-side gather of the accept bitmap: every rank passes the codes
    of its shard (shard(total, rank, world)); rank 0 gets the bitmap of
    all `total` signatures in index order (bit i = code i == 0), other
    ranks None."""
    ok = np.asarray(codes) == 0
    if dist is None:
        return np.packbits(ok, bitorder="little")
    import torch
    world, rank = dist.get_world_size(), dist.get_rank()
    cap = max(hi - lo for lo, hi in (shard(total, r, world) for r in range(world)))
    mine = torch.zeros(cap, dtype=torch.uint8, device=device)
    mine[:len(ok)] = torch.from_numpy(ok.astype(np.uint8)).to(device)
    parts = [torch.zeros(cap, dtype=torch.uint8, device=device) for _ in range(world)]
    dist.all_gather(parts, mine)
    if rank != 0:
        return None
    full = np.concatenate([parts[r].cpu().numpy()[:hi - lo] for r, (lo, hi) in
                           enumerate(shard(total, r, world) for r in range(world))])
    return np.packbits(full.astype(bool), bitorder="little")
