"""The verify tile (include/fd_verify_tile.h):
HA dedup (tcache) semantics against the reference's FD_TCACHE_INSERT
(compiled from src/tango/tcache/fd_tcache.h into oracle/_ref), and on the
GPU a stream of QUIC-format frags (multi-signature txns, corrupted
signatures, HA duplicates, malformed trailers) whose publish decisions,
order and diagnostic counters must equal the reference's per-frag
semantics (src/app/frank/load/fd_frank_verify_synth_load.c:360-410) with
every signature checked by the reference's own fd_ed25519_verify."""
import ctypes

import numpy as np
import pytest

import firedancer_amd as fa
from conftest import oracle_batch
from firedancer_amd import corpus, txn
from firedancer_amd.tile import TCache, VerifyTile


def _ref_tc(ref, depth, map_cnt):
    ref.ref_tcache_new.restype = ctypes.c_void_p
    ref.ref_tcache_new.argtypes = [ctypes.c_ulong, ctypes.c_ulong]
    ref.ref_tcache_insert.argtypes = [ctypes.c_void_p, ctypes.c_ulong]
    ref.ref_tcache_insert.restype = ctypes.c_int
    ref.ref_tcache_delete.argtypes = [ctypes.c_void_p]
    return ref.ref_tcache_new(depth, map_cnt)


@pytest.mark.parametrize("depth,map_cnt", [(16, 64), (1, 4), (4, 8), (100, 256), (30, 32)])
def test_tcache_vs_reference(ref, depth, map_cnt):
    rng = np.random.default_rng(depth * 7 + map_cnt)
    pool = rng.integers(1, 2**63, 3 * depth + 5, dtype=np.int64).astype(np.uint64)
    # collide on the reference's probe start too (low bits equal)
    pool[: depth // 2] = (pool[: depth // 2] & ~np.uint64(map_cnt - 1)) | np.uint64(3)
    tags = rng.choice(pool, 20000)
    tags[rng.random(20000) < 0.01] = 0          # FD_TCACHE_TAG_NULL
    r = _ref_tc(ref, depth, map_cnt)
    ours = TCache(depth, map_cnt)
    for t in tags.tolist():
        assert ours.insert(t) == bool(ref.ref_tcache_insert(r, t)), t
    ref.ref_tcache_delete(r)


def test_tcache_geometry_checked():
    with pytest.raises(ValueError):
        TCache(16, 17)          # not a power of two
    with pytest.raises(ValueError):
        TCache(16, 16)          # map must hold depth + 2


def test_tile_needs_engine():
    assert fa.lib().fd_verify_tile_new(None, None, None, None) is None


def make_stream(n_sigs, seed, ref):
    """-> (frags, per-frag expected (dup, pass)) for a multi-signature stream."""
    b = corpus.solana_txns(n_sigs, seed=seed, sig_dist=[1 / 12] * 12)
    rng = np.random.default_rng(seed)
    starts = sorted({int(d["sig_off"]) // corpus.TXN_MTU * corpus.TXN_MTU for d in b.desc})
    payloads = [bytearray(b.blob[s:s + corpus.TXN_MTU]) for s in starts]
    for p in payloads:                     # ~15% txns: one bad signature (R or S byte)
        if rng.random() < 0.15:
            k = p[0]
            j = int(rng.integers(0, k))
            p[1 + 64 * j + int(rng.integers(8, 64))] ^= 1 << int(rng.integers(0, 8))
    frags = []
    for i, p in enumerate(payloads):
        frags.append(txn.frag(bytes(p)))
        u = rng.random()
        if u < 0.05:
            frags.append(frags[-1])        # immediate HA duplicate
        elif u < 0.08 and i > 40:
            frags.append(txn.frag(bytes(payloads[i - int(rng.integers(1, 40))])))  # near or outside the window
        elif u < 0.10:
            frags.append(frags[-1][:-3] + b"\xff\xff")      # malformed trailer
    return frags


def expected_for(frags, ref):
    """(published (tag, frag) in order, diag counters) frag by frag with the
    reference's tcache and fd_ed25519_verify
    (fd_frank_verify_synth_load.c:360-410)"""
    r = _ref_tc(ref, 16, 64)
    exp_pub, exp = [], dict(HA_FILT_CNT=0, HA_FILT_SZ=0, SV_FILT_CNT=0, SV_FILT_SZ=0, BAD_CNT=0)
    blob, descs, owners, cand = [], [], [], []
    off = 0
    for fi, f in enumerate(frags):
        psz = int.from_bytes(f[-2:], "little")
        t = txn.parse(f[:psz]) if psz <= len(f) - 2 else None
        if t is None or psz > txn.TXN_MTU:
            exp["BAD_CNT"] += 1
            continue
        tag = int.from_bytes(f[t["signature_off"]:t["signature_off"] + 8], "little")
        if ref.ref_tcache_insert(r, tag):
            exp["HA_FILT_CNT"] += 1
            exp["HA_FILT_SZ"] += len(f)
            continue
        d = txn.descs_for(f[:psz], off)
        blob.append(f)
        descs.append(d)
        owners += [len(cand)] * len(d)
        cand.append((tag, f))
        off += len(f)
    ref.ref_tcache_delete(r)
    bb = corpus.Batch(np.frombuffer(b"".join(blob) + b"\0" * 64, np.uint8).copy(), np.concatenate(descs))
    codes = oracle_batch(ref, bb)
    ok = np.ones(len(cand), bool)
    np.logical_and.at(ok, np.array(owners), codes == 0)
    for (tag, f), good in zip(cand, ok):
        if good:
            exp_pub.append((tag, f))
        else:
            exp["SV_FILT_CNT"] += 1
            exp["SV_FILT_SZ"] += len(f)
    return exp_pub, exp, len(codes)


@pytest.mark.gpu
@pytest.mark.parametrize("batch_sigs", [256, 4096])
def test_tile_stream_vs_reference(engine, ref, batch_sigs):
    frags = make_stream(6000, 21 + batch_sigs, ref)
    exp_pub, exp, nsig = expected_for(frags, ref)
    assert 0 < exp["SV_FILT_CNT"] and 0 < exp["HA_FILT_CNT"] and 0 < exp["BAD_CNT"]

    tile = VerifyTile(engine, batch_sigs=batch_sigs)
    for i, f in enumerate(frags):
        tile.rx(f, ctl=i, tsorig=1000 + i)
        if i % 97 == 0:
            tile.service()
    tile.service(flush=True)
    got = [(s, f) for s, f, _, _ in tile.published]
    assert got == exp_pub
    ctl = [c for _, _, c, _ in tile.published]
    assert ctl == sorted(ctl)                                  # published in arrival order
    assert all(ts == 1000 + c for _, _, c, ts in tile.published)
    d = tile.diag()
    for k, v in exp.items():
        assert d[k] == v, k
    assert d["PUB_CNT"] == len(exp_pub) and d["SIG_CNT"] == nsig
    tile.close()


@pytest.mark.gpu
def test_tile_burst_counts_only(engine):
    b = corpus.solana_txns(20000, seed=5, sig_dist=[1 / 12] * 12)
    starts = sorted({int(d["sig_off"]) // corpus.TXN_MTU * corpus.TXN_MTU for d in b.desc})
    frags = [txn.frag(bytes(b.blob[s:s + corpus.TXN_MTU])) for s in starts]
    base = np.frombuffer(b"".join(frags), np.uint8).copy()
    sz = np.array([len(f) for f in frags], np.uint32)
    off = np.concatenate([[0], np.cumsum(sz)[:-1]]).astype(np.uint64)
    tile = VerifyTile(engine, batch_sigs=8192, collect=False)
    tile.rx_burst(base, off, sz)
    tile.service(flush=True)
    d = tile.diag()
    assert d["PUB_CNT"] == len(frags) and d["SIG_CNT"] == 20000 and d["SV_FILT_CNT"] == 0
    assert d["BATCH_CNT"] >= 3
    tile.close()


@pytest.mark.gpu
def test_tile_multi_engine_vs_reference(ref):
    """The multi-engine feeder mode (fd_verify_tile_new_multi) with three
    engines on this box's GPU: every batch goes through an engine's feeder,
    publishes and counters equal the reference's per-frag semantics, in
    arrival order"""
    frags = make_stream(6000, 333, ref)
    exp_pub, exp, nsig = expected_for(frags, ref)
    engines = [fa.Engine(0, 1024, 4 << 20, depth=2) for _ in range(3)]
    try:
        tile = VerifyTile(engines, batch_sigs=512)
        for i, f in enumerate(frags):
            tile.rx(f, ctl=i, tsorig=1000 + i)
            if i % 61 == 0:
                tile.service()
        tile.service(flush=True)
        assert [(s, f) for s, f, _, _ in tile.published] == exp_pub
        ctl = [c for _, _, c, _ in tile.published]
        assert ctl == sorted(ctl)
        d = tile.diag()
        for k, v in exp.items():
            assert d[k] == v, k
        assert d["PUB_CNT"] == len(exp_pub) and d["SIG_CNT"] == nsig and d["BATCH_CNT"] >= 3
        tile.close()
    finally:
        for e in engines:
            e.close()


@pytest.mark.gpu
@pytest.mark.parametrize("batch_sigs,max_blob,engines", [(512, 4 << 20, 1), (4096, 200_000, 1), (512, 300_000, 3)])
def test_tile_inplace_vs_reference(ref, batch_sigs, max_blob, engines):
    """The in-place mode (fd_verify_tile_new_inplace): frags live in one
    registered region (the input dcache's stand-in) and each batch is DMA'd
    from its span there, no copy.  The stream is fed in two passes over two
    halves placed in reverse address order (the second half first), so the
    caller's ring "wraps" to a lower address once: the batch open at the
    wrap continues as a second span (fd_ed25519_gpu_try_submit2, two DMA
    pieces) and the batches equal those of the same stream laid out
    contiguously; a small max_blob closes batches on span size.  Publishes and counters
    equal the reference's per-frag semantics, in arrival order.  With
    engines > 1 the tile runs the multi-engine feeder mode in place
    (fd_verify_tile_new_multi_inplace: the one region registered with
    every engine, round-robin batches through their feeders)."""
    frags = make_stream(6000, 444 + batch_sigs, ref)
    exp_pub, exp, nsig = expected_for(frags, ref)
    h = len(frags) // 2
    first, second = frags[:h], frags[h:]
    # region layout: [second half | first half]; arrival order: first, then second
    lay = second + first
    sz = np.array([len(f) for f in lay], np.uint32)
    off = np.concatenate([[0], np.cumsum(sz)[:-1]]).astype(np.uint64)
    region = np.frombuffer(b"".join(lay) + b"\0" * 64, np.uint8).copy()
    order = list(range(len(second), len(lay))) + list(range(len(second)))
    es = [fa.Engine(0, batch_sigs, max_blob, depth=3 if engines == 1 else 2) for _ in range(engines)]
    try:
        # max_wait_ns=-1: batches close on size only, so the two layouts below
        # can be compared batch for batch (the wait bound is timing-dependent)
        tile = VerifyTile(es[0] if engines == 1 else es, batch_sigs=batch_sigs, region=region, max_wait_ns=-1)
        o, s_ = off[order], sz[order]
        for a in range(0, len(order), 97):                 # bursts, with housekeeping between
            tile.rx_burst(region, o[a:a + 97], s_[a:a + 97], ctl=np.arange(a, min(a + 97, len(order)), dtype=np.uint64))
            tile.service()
            # nothing below the watermark is read again; an open batch holds its frags
            h = tile.held()
            assert h <= min(a + 97, len(order))
            if tile.diag()["BATCH_CNT"] == 0:
                assert h == 0
        tile.service(flush=True)
        assert tile.held() == len(order)
        got = [(s, f) for s, f, _, _ in tile.published]
        assert got == exp_pub
        ctl = [c for _, _, c, _ in tile.published]
        assert ctl == sorted(ctl)
        d = tile.diag()
        for k, v in exp.items():
            assert d[k] == v, k
        assert d["PUB_CNT"] == len(exp_pub) and d["SIG_CNT"] == nsig and d["BATCH_CNT"] >= 3
        # a frag outside the region is malformed input, not a crash
        other = np.frombuffer(frags[0], np.uint8).copy()
        tile.rx_burst(other, np.zeros(1, np.uint64), np.array([len(other)], np.uint32))
        assert tile.diag()["BAD_CNT"] == exp["BAD_CNT"] + 1
        tile.close()
        # the wrap no longer closes a batch: the batch open at the wrap
        # continues as a second span (two DMA pieces), so the same stream
        # laid out contiguously gives the same batches
        lay2 = first + second
        sz2 = np.array([len(f) for f in lay2], np.uint32)
        off2 = np.concatenate([[0], np.cumsum(sz2)[:-1]]).astype(np.uint64)
        region2 = np.frombuffer(b"".join(lay2) + b"\0" * 64, np.uint8).copy()
        tile2 = VerifyTile(es[0] if engines == 1 else es, batch_sigs=batch_sigs, region=region2, max_wait_ns=-1)
        for a in range(0, len(lay2), 97):
            tile2.rx_burst(region2, off2[a:a + 97], sz2[a:a + 97], ctl=np.arange(a, min(a + 97, len(lay2)), dtype=np.uint64))
            tile2.service()
        tile2.service(flush=True)
        assert [(s2, f2) for s2, f2, _, _ in tile2.published] == exp_pub
        assert tile2.diag()["BATCH_CNT"] == d["BATCH_CNT"], (tile2.diag()["BATCH_CNT"], d["BATCH_CNT"])
        tile2.close()
    finally:
        for e in es:
            e.close()
