"""Multi-GPU replica plumbing at world size 2 over gloo on the CPU
(SURVEY.md section 8e): sharding covers every signature once, the timed
region is max-over-ranks, the accept-bitmap gather is index-ordered; and
on the GPU the multi-device dispatcher (several engines, here on one
device) gives the same codes as the reference."""
import os
import socket
import time

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import firedancer_amd as fa
from conftest import oracle_batch
from firedancer_amd import corpus
from firedancer_amd.replicas import gather_bitmap, shard, timed_steps

TOTAL = 1003


def _codes(total):
    rng = np.random.default_rng(1)
    return rng.choice(np.array([0, 0, 0, -1, -2, -3], np.int32), total)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = shard(TOTAL, rank, world)
    codes = _codes(TOTAL)[lo:hi]
    el = timed_steps(lambda: time.sleep(0.05 * (rank + 1)), 2, dist=dist)
    bm = gather_bitmap(codes, TOTAL, dist=dist)
    q.put((rank, lo, hi, el, None if bm is None else bm.tobytes()))
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shards_partition():
    for world in (1, 2, 3, 8):
        rs = [shard(TOTAL, r, world) for r in range(world)]
        assert rs[0][0] == 0 and rs[-1][1] == TOTAL
        assert all(rs[i][1] == rs[i + 1][0] for i in range(world - 1))


def test_gloo_world2_timing_and_gather():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, lo0, hi0, el0, bm0), (_, lo1, hi1, el1, bm1) = res
    assert (lo0, hi1) == (0, TOTAL) and hi0 == lo1
    assert el0 == el1 and el0 >= 2 * 0.1            # max over ranks (rank 1 sleeps 0.1 s/step)
    assert bm1 is None
    exp = np.packbits(_codes(TOTAL) == 0, bitorder="little").tobytes()
    assert bm0 == exp


def test_bitmap_native_matches():
    c = _codes(TOTAL)
    assert fa.codes_to_bitmap(c).tobytes() == np.packbits(c == 0, bitorder="little").tobytes()


def test_multi_fails_loudly_without_gpu():
    if fa.device_count() > 0:
        pytest.skip("a gfx950 device is present")
    with pytest.raises(fa.EngineError):
        fa.MultiEngine([0, 1])


@pytest.mark.gpu
@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0]])
def test_multi_engine_vs_reference(ref, devices):
    b = corpus.concat([corpus.adversarial(3000, 200, seed=len(devices), invalid_frac=0.3),
                       corpus.solana_txns(3000, seed=9, sig_dist=[1 / 12] * 12)])
    m = fa.MultiEngine(devices, max_sigs=1024, max_blob=1 << 20)   # forces several chunks per shard
    got = m.verify_packed(b.blob, b.desc)
    assert (got == oracle_batch(ref, b)).all()
    bad = b.desc.copy()
    bad["msg_sz"][5] = 1 << 30                                      # out of bounds -> ERR_ARG
    got2 = m.verify_packed(b.blob, bad)
    assert got2[5] == fa.ERR_ARG and (np.delete(got2, 5) == np.delete(got, 5)).all()
    m.close()
