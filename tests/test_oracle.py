"""The oracle itself: pinned against the reference's own known answers
and, where the reference build is present, against the reference
compiled from its sources (oracle/_ref/libfdref.so)."""
import ctypes
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, P, ed_vectors, load_corpus, malleability, oracle_batch

L_ORDER = 2**252 + 27742317777372353535851937790883648493


def sha(oracle, msg: bytes) -> bytes:
    out = ctypes.create_string_buffer(64)
    oracle.oracle_sha512(bytes(msg) or b"\0", ctypes.c_uint64(len(msg)), out)
    return out.raw


@pytest.fixture(scope="module")
def shavec():
    return json.load(open(os.path.join(GOLDEN, "sha512_vectors.json")))


def test_sha512_cavp_short(oracle, shavec):
    for v in shavec["cavp_short"]:
        assert sha(oracle, bytes.fromhex(v["msg"])).hex() == v["md"]


def test_sha512_cavp_long(oracle, shavec):
    for v in shavec["cavp_long"]:
        assert sha(oracle, bytes.fromhex(v["msg"])).hex() == v["md"]


def test_sha512_cavp_monte(oracle, shavec):
    # FIPS 180-4 SHAVS Monte Carlo: MD_i = SHA(MD_{i-3} || MD_{i-2} || MD_{i-1})
    seed = bytes.fromhex(shavec["cavp_monte"]["seed"])
    for j, expect in enumerate(shavec["cavp_monte"]["md"][:20]):
        md = [seed, seed, seed]
        for _ in range(1000):
            md = [md[1], md[2], sha(oracle, md[0] + md[1] + md[2])]
        seed = md[2]
        assert seed.hex() == expect, j


def test_sha512_fd_vectors(oracle, shavec):
    assert len(shavec["fd_test_vector"]) == 45
    for v in shavec["fd_test_vector"]:
        assert sha(oracle, bytes.fromhex(v["msg"])).hex() == v["md"]


def test_sc_reduce_canonical(oracle):
    rng = np.random.default_rng(1)
    edge = [b"\0" * 64, b"\xff" * 64, L_ORDER.to_bytes(64, "little"), (L_ORDER - 1).to_bytes(64, "little"),
            (L_ORDER + 1).to_bytes(64, "little"), (2 * L_ORDER).to_bytes(64, "little"),
            (L_ORDER * (2**259 - 1)).to_bytes(64, "little")]
    ins = edge + [rng.bytes(64) for _ in range(4000)]
    for x in ins:
        out = ctypes.create_string_buffer(32)
        oracle.oracle_sc_reduce(x, out)
        assert int.from_bytes(out.raw, "little") == int.from_bytes(x, "little") % L_ORDER


def test_sc_reduce_vs_reference(oracle, ref):
    rng = np.random.default_rng(2)
    for _ in range(2000):
        x = rng.bytes(64)
        a, b = ctypes.create_string_buffer(32), ctypes.create_string_buffer(32)
        oracle.oracle_sc_reduce(x, a)
        ref.ref_sc_reduce(x, b)
        assert a.raw == b.raw


def _rand_fe(rng, n, bits=26):
    v = rng.integers(-(1 << (bits - 1)), 1 << (bits - 1), (n, 10), dtype=np.int64).astype(np.int32)
    return v


def test_field_ops_vs_reference(oracle, ref):
    rng = np.random.default_rng(3)
    for bits in (25, 26, 27):
        F, G = _rand_fe(rng, 3000, bits), _rand_fe(rng, 3000, bits)
        for f, g in zip(F, G):
            f = np.ascontiguousarray(f); g = np.ascontiguousarray(g)
            for fn in ("fe_mul_avx", "fe_mul_scalar"):
                a, b = np.zeros(10, np.int32), np.zeros(10, np.int32)
                getattr(oracle, "oracle_" + fn)(P(a), P(f), P(g))
                getattr(ref, "ref_" + fn)(P(b), P(f), P(g))
                assert (a == b).all(), fn
            for n in (1, 2):
                a, b = np.zeros(10, np.int32), np.zeros(10, np.int32)
                oracle.oracle_fe_sqn_avx(P(a), P(f), n)
                ref.ref_fe_sqn_avx(P(b), P(f), n)
                assert (a == b).all()


def test_frombytes_tobytes_vs_reference(oracle, ref):
    rng = np.random.default_rng(4)
    for _ in range(3000):
        s = rng.bytes(32)
        a, b = np.zeros(10, np.int32), np.zeros(10, np.int32)
        oracle.oracle_fe_frombytes(P(a), s)
        ref.ref_fe_frombytes(P(b), s)
        assert (a == b).all()
        f = _rand_fe(rng, 1, 26)[0]
        x, y = ctypes.create_string_buffer(32), ctypes.create_string_buffer(32)
        oracle.oracle_fe_tobytes(x, P(f))
        ref.ref_fe_tobytes(y, P(f))
        assert x.raw == y.raw


def test_group_ops_vs_reference(oracle, ref):
    """decompression, small-order test and the double-scalar multiplication,
    limb-for-limb, on random and on small-order / off-curve encodings."""
    from firedancer_amd import corpus
    rng = np.random.default_rng(5)
    encs = [rng.bytes(32) for _ in range(600)] + corpus.small_order_encodings()
    for i in range(0, len(encs) - 1, 2):
        a0, a1 = np.zeros(40, np.int32), np.zeros(40, np.int32)
        r0, r1 = np.zeros(40, np.int32), np.zeros(40, np.int32)
        e_ref = ref.ref_ge_frombytes_2(P(r0), encs[i], P(r1), encs[i + 1])
        e0 = oracle.oracle_ge_frombytes(P(a0), encs[i])
        e1 = oracle.oracle_ge_frombytes(P(a1), encs[i + 1])
        assert e_ref == (e0 or e1)
        if e_ref == 0:
            assert (a0 == r0).all() and (a1 == r1).all()
            for pt in (a0, a1):
                assert oracle.oracle_ge_is_small_order(P(pt)) == ref.ref_ge_is_small_order(P(pt))
                ka, kb = rng.bytes(32), bytearray(rng.bytes(32))
                kb[31] &= 0x0F
                o1, o2 = np.zeros(30, np.int32), np.zeros(30, np.int32)
                oracle.oracle_ge_dsm(P(o1), ka, P(pt), bytes(kb))
                ref.ref_ge_dsm(P(o2), ka, P(pt), bytes(kb))
                assert (o1 == o2).all()


def test_slide_properties(oracle):
    """the signed digits reconstruct the scalar and are odd in [-15,15]"""
    rng = np.random.default_rng(6)
    for _ in range(500):
        a = bytearray(rng.bytes(32))
        a[31] &= 0x1F
        r = np.zeros(256, np.int8)
        oracle.oracle_ge_slide(P(r), bytes(a))
        assert sum(int(d) << i for i, d in enumerate(r)) == int.from_bytes(a, "little")
        nz = r[r != 0]
        assert ((nz % 2) != 0).all() and (np.abs(nz) <= 15).all()


@pytest.mark.parametrize("name", ["adversarial", "txn1232", "small_order", "msgsizes"])
def test_oracle_golden_corpora(oracle, name):
    b, exp = load_corpus(name)
    got = oracle_batch(oracle, b)
    assert (got == exp).all(), np.nonzero(got != exp)[0][:20]


def test_oracle_vectors(oracle):
    for v in ed_vectors():
        m = bytes.fromhex(v["msg"])
        got = oracle.oracle_verify(m or b"\0", len(m), bytes.fromhex(v["sig"]), bytes.fromhex(v["pub"]))
        assert got == v["expected"], v["name"]


def test_oracle_malleability(oracle):
    """test_ed25519_signature_malleability.c: 200 must pass, 196 must fail"""
    for sig, pub, ok in malleability():
        got = oracle.oracle_verify(b"Zcash", 5, sig, pub)
        assert (got == 0) == ok


def test_oracle_vs_reference_random(oracle, ref):
    from firedancer_amd import corpus
    b = corpus.adversarial(8000, 200, seed=77, invalid_frac=0.3)
    assert (oracle_batch(oracle, b) == oracle_batch(ref, b)).all()
