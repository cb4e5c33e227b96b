"""GPU parity: every per-signature code of the engine equals the
reference's (AVX2 fd_ed25519_verify) on the same inputs.

Checkers: the committed golden corpora (expected codes produced by the
reference build), the reference build itself when it was shipped with
the tree (oracle/_ref/libfdref.so), and the CPU restatement
(oracle/liboracle.so).  Full BASELINE sizes are covered through
size-independent properties (all-valid => all accept, permutation
equivariance, repeatability, corruption => reject)."""
import ctypes
import os

import numpy as np
import pytest

import firedancer_amd as fa
from conftest import ROOT, ed_vectors, load_corpus, malleability, oracle_batch
from firedancer_amd import corpus, txn

pytestmark = pytest.mark.gpu


def _checker(ref):
    """the reference build itself (the `ref` fixture fails when it is absent)"""
    return ref


@pytest.mark.parametrize("name", ["adversarial", "txn1232", "small_order", "msgsizes"])
def test_golden_corpora(engine, name):
    b, exp = load_corpus(name)
    got = engine.verify_packed(b.blob, b.desc)
    bad = np.nonzero(got != exp)[0]
    assert len(bad) == 0, [(int(i), int(exp[i]), int(got[i])) for i in bad[:10]]


def test_vectors_rfc8032_and_q2(engine):
    vs = ed_vectors()
    b = corpus.from_triples([(bytes.fromhex(v["msg"]), bytes.fromhex(v["sig"]), bytes.fromhex(v["pub"])) for v in vs])
    got = engine.verify_packed(b.blob, b.desc)
    assert got.tolist() == [v["expected"] for v in vs]
    # the three Q2 vectors are valid RFC 8032 signatures the reference rejects
    assert got[-3:].tolist() == [-3, -3, -3]


def test_malleability_kats(engine):
    m = malleability()
    b = corpus.from_triples([(b"Zcash", s, p) for s, p, _ in m])
    got = engine.verify_packed(b.blob, b.desc)
    for (s, p, ok), g in zip(m, got):
        assert (g == 0) == ok


def test_txn_fixtures(engine):
    from conftest import GOLDEN
    parts, descs, off = [], [], 0
    for i in (1, 2, 3):
        p = open(os.path.join(GOLDEN, f"transaction{i}.bin"), "rb").read()
        descs.append(txn.descs_for(p, off))
        parts.append(p)
        off += len(p)
    blob = np.frombuffer(b"".join(parts) + b"\0" * 64, np.uint8).copy()
    got = engine.verify_packed(blob, np.concatenate(descs))
    assert got.tolist() == [0] * 6


def test_adversarial_vs_reference(engine, ref):
    """C3 shape at 64K signatures, 10% invalid, checked signature by
    signature against the reference build."""
    chk = _checker(ref)
    b = corpus.adversarial(65536, 128, seed=2024, invalid_frac=0.1)
    exp = oracle_batch(chk, b)
    got = engine.verify_packed(b.blob, b.desc)
    bad = np.nonzero(got != exp)[0]
    assert len(bad) == 0, [(int(i), corpus.CASES[b.label[i]], int(exp[i]), int(got[i])) for i in bad[:10]]


def test_txn_mtu_batches_vs_reference(engine, ref):
    """C2 shape: 4096-signature batches of 1232-byte txns, 1-2 sigs each,
    with 5% of signatures corrupted."""
    chk = _checker(ref)
    b = corpus.solana_txns(4096 * 4, seed=77)
    rng = np.random.default_rng(5)
    for i in rng.choice(len(b), len(b) // 20, replace=False):
        b.blob[int(b.desc[i]["sig_off"]) + rng.integers(0, 64)] ^= np.uint8(1 << rng.integers(0, 8))
    exp = oracle_batch(chk, b)
    got = engine.verify_packed(b.blob, b.desc)
    assert (got == exp).all()
    assert (exp != 0).sum() > 0


def test_full_size_properties(engine):
    """BASELINE C2 at full batch size (64 x 4096 signatures): all valid
    => all accepted; permuting descriptors permutes results; two runs
    agree; flipping one byte of each of 512 signatures rejects them."""
    base = corpus.solana_txns(16384, seed=31)
    b = base.tile(16)
    got = engine.verify_packed(b.blob, b.desc)
    assert (got == 0).all()
    perm = np.random.default_rng(1).permutation(len(b))
    got_p = engine.verify_packed(b.blob, b.desc[perm])
    assert (got_p == got[perm]).all()
    blob = base.blob.copy()
    idx = np.random.default_rng(2).choice(len(base), 512, replace=False)
    for i in idx:
        blob[int(base.desc[i]["sig_off"]) + 40] ^= 0x01   # S byte 8
    got2 = engine.verify_packed(blob, base.desc)
    assert (got2[idx] != 0).all()
    mask = np.ones(len(base), bool)
    mask[idx] = False
    # only the corrupted signatures (and co-signers sharing nothing) change
    assert (got2[mask] == 0).all()


def test_empty_and_single(engine):
    out = engine.verify_packed(np.zeros(64, np.uint8), np.zeros(0, fa.DESC_DTYPE))
    assert len(out) == 0
    b = corpus.simple(1, 0, seed=3)
    assert engine.verify_packed(b.blob, b.desc).tolist() == [0]


def test_malformed_descriptors(engine):
    b = corpus.simple(8, 64, seed=4)
    d = b.desc.copy()
    d[3]["msg_sz"] = 1 << 30          # message runs past the blob
    d[5]["sig_off"] = len(b.blob)      # signature outside the blob
    got = engine.verify_packed(b.blob, d)
    assert got[3] == fa.ERR_ARG and got[5] == fa.ERR_ARG
    assert (np.delete(got, [3, 5]) == 0).all()


def test_reference_shaped_apis(engine):
    """fd_ed25519_verify, fd_ed25519_verify_batch and
    fd_ed25519_verify_batch_single_msg on the process-default engine."""
    b = corpus.adversarial(600, 100, seed=8, invalid_frac=0.3)
    exp = engine.verify_packed(b.blob, b.desc)
    msgs = [b.msg(i) for i in range(len(b))]
    sigs = [b.sig(i) for i in range(len(b))]
    pubs = [b.pub(i) for i in range(len(b))]
    r, out = fa.verify_batch(msgs, sigs, pubs)
    assert (out == exp).all()
    first = exp[exp != 0]
    assert r == (int(first[0]) if len(first) else 0)
    for i in range(0, 600, 37):
        assert fa.verify(msgs[i], sigs[i], pubs[i]) == exp[i]
    # vote-shaped: many signers over one 442-byte message (transaction2 size)
    sb, msg, sig, pub = corpus.single_msg(4096, 442, seed=9)
    r, out = fa.verify_batch_single_msg(bytes(msg), sig, pub)
    assert r == 0 and (out == 0).all()
    sig2 = sig.copy()
    sig2[100, 0] ^= 1
    r, out = fa.verify_batch_single_msg(bytes(msg), sig2, pub)
    assert out[100] != 0 and r == out[100] and (np.delete(out, 100) == 0).all()


def test_per_signature_calls_concurrent(engine, ref):
    """fd_ed25519_verify from 16 threads at once: the calls coalesce into
    shared batches on the process-default engine (group commit), and every
    call still returns its own signature's code, equal to the reference's;
    a call with a message larger than the engine's 64 MiB staging blob
    takes the long path (device SHA-512 in pieces) and gets the reference's
    code, without failing the calls it shares a batch with."""
    import threading
    b = corpus.adversarial(16 * 48, 100, seed=18, invalid_frac=0.3)
    exp = oracle_batch(ref, b)
    msgs = [b.msg(i) for i in range(len(b))]
    sigs = [b.sig(i) for i in range(len(b))]
    pubs = [b.pub(i) for i in range(len(b))]
    got = np.full(len(b), 99, np.int32)
    big = [None]

    def worker(t):
        for i in range(t, len(b), 16):
            got[i] = fa.verify(msgs[i], sigs[i], pubs[i])
        if t == 0:
            big[0] = fa.verify(bytes(1 << 27), sigs[0], pubs[0])
    th = [threading.Thread(target=worker, args=(t,)) for t in range(16)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert (got == exp).all()
    bm = np.zeros(1 << 27, np.uint8)
    assert big[0] == ref.ref_verify(bm.ctypes.data, len(bm), sigs[0], pubs[0])


def test_async_ring(engine):
    """submit/poll over the pinned ring: depth batches in flight, each
    result identical to the synchronous path."""
    bs = [corpus.adversarial(2048, 128, seed=40 + k, invalid_frac=0.2) for k in range(engine.depth)]
    exp = [engine.verify_packed(b.blob, b.desc) for b in bs]
    tickets = [engine.submit(b.blob, b.desc) for b in bs]
    for t, b, e in zip(tickets, bs, exp):
        out = np.zeros(len(b), np.int32)
        assert engine.poll(t, out, block=True)
        assert (out == e).all()


def test_ring_cu_groups_vs_reference(engine, ref):
    """Small batches kept in flight at full ring depth run on their slots'
    CU groups (fd_ed25519_gpu_host.cpp): 4 x depth 4096-signature
    adversarial batches through submit/poll, every code checked against
    the reference build."""
    chk = _checker(ref)
    b = corpus.adversarial(4096 * 2, 128, seed=99, invalid_frac=0.2)
    exp = oracle_batch(chk, b)
    halves = []
    for h in range(2):
        d = b.desc[h * 4096:(h + 1) * 4096].copy()
        halves.append((b.blob, d, exp[h * 4096:(h + 1) * 4096]))
    inflight = []
    out = np.zeros(4096, np.int32)
    for k in range(4 * engine.depth):
        if len(inflight) == engine.depth:
            t, e = inflight.pop(0)
            assert engine.poll(t, out, block=True)
            assert (out == e).all()
        blob, d, e = halves[k % 2]
        inflight.append((engine.submit(blob, d), e))
    for t, e in inflight:
        assert engine.poll(t, out, block=True)
        assert (out == e).all()


def test_device_resident(engine):
    """verify_dev on torch-allocated HBM (the bench's path)."""
    torch = pytest.importorskip("torch")
    b = corpus.adversarial(4096, 128, seed=12, invalid_frac=0.2)
    exp = engine.verify_packed(b.blob, b.desc)
    blob = torch.from_numpy(np.concatenate([b.blob, np.zeros(64, np.uint8)])).cuda()
    desc = torch.from_numpy(b.desc.view(np.uint8).copy()).cuda()
    out = torch.zeros(len(b), dtype=torch.int32, device="cuda")
    engine.verify_dev(len(b), blob.data_ptr(), len(b.blob), desc.data_ptr(), out.data_ptr(),
                      torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert (out.cpu().numpy() == exp).all()


@pytest.fixture(scope="module")
def pooled():
    """an engine that runs the pooled DSM (fd_k_dsm_pool) for every batch"""
    e = fa.Engine(0, 1 << 18, 1 << 28)
    e.dsm_pool_min = 0
    yield e
    e.close()


@pytest.mark.parametrize("name", ["adversarial", "txn1232", "small_order", "msgsizes"])
def test_pooled_dsm_golden_corpora(pooled, name):
    """the pooled schedule steps signatures in a data-dependent order; the
    codes must still be the reference's"""
    b, exp = load_corpus(name)
    got = pooled.verify_packed(b.blob, b.desc)
    bad = np.nonzero(got != exp)[0]
    assert len(bad) == 0, [(int(i), int(exp[i]), int(got[i])) for i in bad[:10]]


@pytest.mark.parametrize("n", [1, 63, 129, 4096 + 77, 40000])
def test_pooled_equals_uniform(engine, pooled, n):
    """ragged pools (n not a multiple of 128, fewer slots than lanes) and
    several waves: pooled and uniform schedules give identical codes on a
    mixed valid / invalid batch"""
    base, _ = load_corpus("adversarial")
    b = base.tile(int(np.ceil(n / len(base))))
    b.desc = b.desc[:n]
    engine.dsm_pool_min = 1 << 62
    engine.dsm_quad_max = engine.dsm_oct_max = 0
    a = engine.verify_packed(b.blob, b.desc)
    p = pooled.verify_packed(b.blob, b.desc)
    assert (a == p).all(), np.nonzero(a != p)[0][:10]
    assert engine.dsm_pool_min == 1 << 62
    engine.dsm_pool_min = 262144
    engine.dsm_quad_max = 32768
    engine.dsm_oct_max = 64


@pytest.mark.parametrize("sizes", [(40000, 4176, 40048, 4163)])
def test_step_major_op_zeroing_vs_reference(pooled, uniform, ref, sizes):
    """step-major op streams (pooled and uniform DSMs) are zero-filled
    before fd_k_prep stores the additions; each batch runs on an op buffer
    the previous, differently strided batch left full of additions (sizes
    with and without a partly live last wave), and its codes must be the
    reference's"""
    base, _ = load_corpus("adversarial")
    for eng in (pooled, uniform):
        for n in sizes:
            b = base.tile(int(np.ceil(n / len(base))))
            b.desc = b.desc[:n]
            got = eng.verify_packed(b.blob, b.desc)
            exp = oracle_batch(ref, b)
            bad = np.nonzero(got != exp)[0]
            assert len(bad) == 0, (n, [(int(i), int(exp[i]), int(got[i])) for i in bad[:10]])


@pytest.fixture(scope="module")
def uniform():
    """an engine that runs the one-lane-per-signature DSM (fd_k_dsm) for
    every batch"""
    e = fa.Engine(0, 1 << 18, 1 << 28)
    e.dsm_pool_min = 1 << 62
    e.dsm_quad_max = e.dsm_oct_max = 0
    yield e
    e.close()


@pytest.mark.parametrize("name", ["adversarial", "txn1232", "small_order", "msgsizes"])
def test_uniform_dsm_golden_corpora(uniform, name):
    b, exp = load_corpus(name)
    got = uniform.verify_packed(b.blob, b.desc)
    bad = np.nonzero(got != exp)[0]
    assert len(bad) == 0, [(int(i), int(exp[i]), int(got[i])) for i in bad[:10]]


@pytest.mark.parametrize("n", [1, 15, 17, 4096 + 77, 30000])
def test_quad_equals_uniform(engine, uniform, n):
    """the quad-lane DSM (fd_k_dsm_quad, the default up to 32768
    signatures) against the uniform one on ragged batches (n not a multiple
    of the 16 signatures of a wave) of mixed valid / invalid signatures"""
    base, _ = load_corpus("adversarial")
    b = base.tile(int(np.ceil(n / len(base))))
    b.desc = b.desc[:n]
    assert engine.dsm_quad_max >= n
    engine.dsm_oct_max = 0              # the quad, also for n <= 64
    try:
        q = engine.verify_packed(b.blob, b.desc)
    finally:
        engine.dsm_oct_max = 64
    u = uniform.verify_packed(b.blob, b.desc)
    assert (q == u).all(), np.nonzero(q != u)[0][:10]


def test_quad_messages_at_every_alignment(engine, uniform):
    """the latency front end (fd_k_front) reads each message at its own byte
    alignment: the same signatures packed with every start offset mod 16 of
    sig, pub and message, through the quad schedule and the uniform one
    (fd_k_prep's front end), all valid.  (A build whose schedule wave lost
    its staging buffer still passed the golden corpora, whose messages sit
    16-aligned, and rejected every unaligned one.)"""
    base = corpus.solana_txns(512, seed=91)
    trip = [(base.msg(i), base.sig(i), base.pub(i)) for i in range(len(base))]
    parts, desc, off = [], np.zeros(len(trip), corpus.DESC_DTYPE), 0
    for i, (m, sg, pb) in enumerate(trip):
        pad = (i * 7) % 16 + (i // 16) % 3          # every residue mod 16, with the fields at mixed offsets
        parts.append(b"\x55" * pad)
        off += pad
        desc[i] = (off, off + 64, off + 96 + (i % 5), len(m))
        parts.append(bytes(sg) + bytes(pb) + b"\xaa" * (i % 5) + bytes(m))
        off += 96 + (i % 5) + len(m)
    blob = np.frombuffer(b"".join(parts) + b"\0" * 64, np.uint8).copy()
    assert len(set((desc["msg_off"] % 16).tolist())) == 16
    assert engine.dsm_quad_max >= len(desc)
    q = engine.verify_packed(blob, desc)
    u = uniform.verify_packed(blob, desc)
    assert (q == 0).all() and (u == 0).all(), (np.nonzero(q)[0][:8], np.nonzero(u)[0][:8])


def test_quad_q2_vectors(engine):
    """the reference-quirk (Q2) and RFC 8032 vectors through the quad
    schedule explicitly"""
    vs = ed_vectors()
    b = corpus.from_triples([(bytes.fromhex(v["msg"]), bytes.fromhex(v["sig"]), bytes.fromhex(v["pub"])) for v in vs])
    assert len(b) <= engine.dsm_quad_max
    engine.dsm_oct_max = 0
    try:
        got = engine.verify_packed(b.blob, b.desc)
    finally:
        engine.dsm_oct_max = 64
    assert got.tolist() == [v["expected"] for v in vs]


@pytest.fixture(scope="module")
def oct():
    """an engine that runs the eight-lane DSM (fd_k_dsm_oct, the default up
    to 64 signatures) for every batch size"""
    e = fa.Engine(0, 1 << 18, 1 << 28)
    e.dsm_pool_min = 1 << 62
    e.dsm_oct_max = 1 << 62
    yield e
    e.close()


@pytest.mark.parametrize("name", ["adversarial", "txn1232", "small_order", "msgsizes"])
def test_oct_dsm_golden_corpora(oct, name):
    b, exp = load_corpus(name)
    got = oct.verify_packed(b.blob, b.desc)
    bad = np.nonzero(got != exp)[0]
    assert len(bad) == 0, [(int(i), int(exp[i]), int(got[i])) for i in bad[:10]]


def test_oct_q2_vectors_and_malleability(engine, oct):
    """the reference-quirk (Q2) and RFC 8032 vectors and the malleability
    KATs through the oct schedule, at its default size (one batch of at most
    64 on the default engine) and forced"""
    vs = ed_vectors()
    b = corpus.from_triples([(bytes.fromhex(v["msg"]), bytes.fromhex(v["sig"]), bytes.fromhex(v["pub"])) for v in vs])
    assert len(b) <= engine.dsm_oct_max
    for e in (engine, oct):
        got = e.verify_packed(b.blob, b.desc)
        assert got.tolist() == [v["expected"] for v in vs]
        assert got[-3:].tolist() == [-3, -3, -3]
    m = malleability()
    bm = corpus.from_triples([(b"Zcash", s, p) for s, p, _ in m])
    for e in (engine, oct):
        got = e.verify_packed(bm.blob, bm.desc)
        for (s, p, ok), g in zip(m, got):
            assert (g == 0) == ok


@pytest.mark.parametrize("n", [1, 7, 9, 63, 64])
def test_oct_equals_uniform_default_sizes(engine, uniform, n):
    """the default engine's small batches (the oct DSM) against the uniform
    DSM on ragged batches (n not a multiple of the 8 signatures of a wave)
    of mixed valid / invalid signatures"""
    base, _ = load_corpus("adversarial")
    b = base.tile(int(np.ceil(n / len(base))))
    b.desc = b.desc[:n]
    assert engine.dsm_oct_max >= n
    o = engine.verify_packed(b.blob, b.desc)
    u = uniform.verify_packed(b.blob, b.desc)
    assert (o == u).all(), np.nonzero(o != u)[0][:10]


@pytest.mark.parametrize("n", [4096 + 77, 30000])
def test_oct_equals_uniform_forced(oct, uniform, n):
    base = corpus.adversarial(n, 200, seed=95 + n, invalid_frac=0.2)
    o = oct.verify_packed(base.blob, base.desc)
    u = uniform.verify_packed(base.blob, base.desc)
    assert (o == u).all(), np.nonzero(o != u)[0][:10]


@pytest.mark.parametrize("n", [1, 5, 32, 33])
def test_small_batches_s_recoded_ahead(engine, ref, n):
    """Batches of at most 32 have S's digits recoded ahead on an idle front-end
    wave (fd_sdig_body) and the prep wave runs only k's pass; S at or above
    2^252 that still passes the range check (S = L - 1 .. L - 3) is skipped
    there and recoded by prep itself, in the same wave as lanes that take
    the digits ahead.  Codes equal the reference's; n = 33 is one past the
    offload."""
    b = corpus.adversarial(n, 150, seed=300 + n, invalid_frac=0.0)
    L = corpus.L
    for j in range(1, n, 4):      # every fourth signature: S just below L
        so = int(b.desc[j]["sig_off"])
        b.blob[so + 32:so + 64] = np.frombuffer((L - 1 - (j % 3)).to_bytes(32, "little"), np.uint8)
    exp = oracle_batch(ref, b)
    for rep in range(3):          # repeated launches reuse the scratch with new tags
        got = engine.verify_packed(b.blob, b.desc)
        assert (got == exp).all(), (rep, np.nonzero(got != exp)[0][:10], got[:8], exp[:8])
    assert (exp == 0).sum() >= n - (n + 2) // 4
