"""Transaction wire parsing: the native
fd_txn_parse (firedancer_amd/csrc/fd_txn_host.c) against the reference
parser compiled in place (oracle/_ref, src/ballet/txn/fd_txn_parse.c) and
against golden results the reference produced (tests/golden/
txn_parse_golden.json, made by tests/golden/make_txn_golden.py).

The differential sweep is the reference's own test_mutate
(src/ballet/txn/test_txn_parse.c:107-190): every truncation and every
single-byte value of every position of each fixture; return value,
descriptor bytes and parse counters (incl. the failure ring of source
lines) must agree exactly."""
import ctypes
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, oracle_batch
from firedancer_amd import corpus, txn

RING = txn.COUNTERS_RING_SZ


def fixtures():
    return [open(os.path.join(GOLDEN, f"transaction{i}.bin"), "rb").read() for i in (1, 2, 3)]


def golden():
    return json.load(open(os.path.join(GOLDEN, "txn_parse_golden.json")))


def _parser(L, name):
    f = getattr(L, name)
    f.argtypes = [ctypes.c_void_p, ctypes.c_ulong, ctypes.c_void_p, ctypes.c_void_p]
    f.restype = ctypes.c_ulong
    return f


def sweep(fn, payload):
    """test_mutate's input set through one parser -> (sha256 of all
    (footprint, descriptor) results, counters)."""
    n = len(payload)
    buf = (ctypes.c_uint8 * n).from_buffer(bytearray(payload))
    out = ctypes.create_string_buffer(txn.TXN_MAX_SZ)
    ctr = txn.Counters()
    h = hashlib.sha256()
    addr, oaddr, cp = ctypes.addressof(buf), ctypes.addressof(out), ctypes.byref(ctr)
    for i in range(n):
        fp = fn(addr, i, oaddr, cp)                      # truncated to i bytes
        h.update(fp.to_bytes(8, "little"))
        orig = buf[i]
        for d in range(1, 256):
            buf[i] = (orig + d) & 0xFF
            fp = fn(addr, n, oaddr, cp)
            h.update(fp.to_bytes(8, "little"))
            if fp:
                h.update(out.raw[:fp])
        buf[i] = orig
    return h.hexdigest(), (ctr.success_cnt, ctr.failure_cnt, list(ctr.failure_ring))


def test_parse_fixtures_fields():
    """src/ballet/txn/test_txn_parse.c:20-105 (txn1/txn2 correctness)."""
    t1, t2, t3 = [txn.parse(p) for p in fixtures()]
    p1, p2 = fixtures()[:2]
    assert (t1["transaction_version"], t1["signature_cnt"]) == (0xFF, 4)
    assert [p1[t1["signature_off"] + 64 * j] for j in range(4)] == [97, 189, 11, 108]
    assert t1["message_off"] == t1["signature_off"] + 4 * 64
    assert (t1["readonly_signed_cnt"], t1["readonly_unsigned_cnt"], t1["acct_addr_cnt"]) == (1, 11, 23)
    assert [p1[t1["acct_addr_off"] + 32 * j] for j in range(23)] == [
        220, 255, 85, 89, 201, 170, 194, 48, 228, 123, 151, 133, 6, 6, 203, 6, 11, 6, 0, 140, 3, 5, 168]
    assert p1[t1["recent_blockhash_off"]] == 155
    assert (t1["addr_table_lookup_cnt"], t1["instr_cnt"]) == (0, 7)
    ix = t1["instr"]
    assert ix[0][0] == 20 and ix[0][2] == 0 and ix[0][3] == 5
    assert p1[ix[0][5]:ix[0][5] + 5] == b"\x00\xE0\x93\x04\x00"
    assert (ix[6][0], ix[6][2], ix[6][3]) == (22, 21, 12)
    assert (p1[ix[6][4]], p1[ix[6][5]]) == (14, 211)
    assert (t2["transaction_version"], t2["signature_cnt"], p2[t2["signature_off"]]) == (0, 1, 184)
    assert (t2["readonly_signed_cnt"], t2["readonly_unsigned_cnt"], t2["acct_addr_cnt"]) == (0, 2, 6)
    assert (t2["addr_table_lookup_cnt"], t2["addr_table_adtl_writable_cnt"], t2["addr_table_adtl_cnt"]) == (3, 12, 21)
    luts = t2["luts"]
    assert p2[luts[0][0]] == 54 and luts[0][1:3] == (4, 4)
    assert p2[luts[0][3]:luts[0][3] + 4] == bytes([142, 141, 143, 144])
    assert p2[luts[2][0]] == 212 and luts[2][1:3] == (4, 1)
    assert t3["footprint"] == len(t3["raw"]) and t3["signature_cnt"] == 1


def test_fixtures_match_golden():
    g = golden()
    for p, exp in zip(fixtures(), g["fixtures"]):
        fp, raw = txn.parse_raw(p)
        assert fp == exp["footprint"] and raw.hex() == exp["raw"]


@pytest.mark.parametrize("k", [0, 1, 2])
def test_mutation_sweep_matches_golden(k):
    digest, ctr = sweep(_parser(txn.lib(), "fd_txn_parse"), fixtures()[k])
    exp = golden()["sweep"][k]
    assert ctr[0] == exp["success_cnt"] and ctr[1] == exp["failure_cnt"]
    assert ctr[2] == exp["failure_ring"]
    assert digest == exp["sha256"]


def test_mutation_sweep_vs_reference(ref):
    ours, theirs = _parser(txn.lib(), "fd_txn_parse"), _parser(ref, "ref_txn_parse")
    for p in fixtures():
        assert sweep(ours, p) == sweep(theirs, p)


def test_random_payloads_vs_reference(ref):
    """Random and synthetic payloads, incl. v0 headers and > 64 KiB."""
    ours, theirs = _parser(txn.lib(), "fd_txn_parse"), _parser(ref, "ref_txn_parse")
    rng = np.random.default_rng(11)
    cands = [bytes(rng.integers(0, 256, int(rng.integers(0, 300)), dtype=np.uint8)) for _ in range(3000)]
    b = corpus.solana_txns(200, seed=4, sig_dist=[1 / 12] * 12, max_sigs_per_txn=12)
    cands += [bytes(b.blob[i * corpus.TXN_MTU:(i + 1) * corpus.TXN_MTU]) for i in range(20)]
    cands += [b"\x01" + b"\x00" * 70000]
    for p in cands:
        c1, c2 = txn.Counters(), txn.Counters()
        o1, o2 = ctypes.create_string_buffer(txn.TXN_MAX_SZ), ctypes.create_string_buffer(txn.TXN_MAX_SZ)
        r1 = ours(p, len(p), o1, ctypes.byref(c1))
        r2 = theirs(p, len(p), o2, ctypes.byref(c2))
        assert r1 == r2 and o1.raw[:r1] == o2.raw[:r2]
        assert (c1.success_cnt, c1.failure_cnt, c1.failure_ring[0]) == (c2.success_cnt, c2.failure_cnt, c2.failure_ring[0])


def test_fixture_signatures_verify(oracle):
    parts, descs, off = [], [], 0
    for p in fixtures():
        descs.append(txn.descs_for(p, off))
        parts.append(p)
        off += len(p)
    b = corpus.Batch(np.frombuffer(b"".join(parts) + b"\0" * 64, np.uint8).copy(), np.concatenate(descs))
    assert len(b) == 6
    assert (oracle_batch(oracle, b) == 0).all()


def test_malformed_rejected():
    p = fixtures()[2]
    assert txn.parse(p[:-1]) is None                 # truncated
    assert txn.parse(b"\x00" + p[1:]) is None        # zero signatures
    assert txn.parse(p + b"\x00") is None            # trailing bytes
    assert txn.parse(b"\x80\x80\x80" + p[3:]) is None  # bad compact-u16
    assert txn.parse(b"") is None


def test_synthetic_txns_parse_and_frag():
    b = corpus.solana_txns(300, seed=3, sig_dist=[1 / 12] * 12, max_sigs_per_txn=12)
    starts = sorted({int(d["sig_off"]) // corpus.TXN_MTU * corpus.TXN_MTU for d in b.desc})
    seen = 0
    for base in starts:
        p = bytes(b.blob[base:base + corpus.TXN_MTU])
        t = txn.parse(p)
        assert t is not None and t["message_off"] == 1 + 64 * t["signature_cnt"]
        d = txn.descs_for(p, base)
        assert (d == b.desc[seen:seen + len(d)]).all()
        seen += len(d)
        f = txn.frag(p)
        assert f[-2:] == len(p).to_bytes(2, "little") and f[:len(p)] == p
        assert f[len(p):len(p) + t["footprint"]] == t["raw"]
    assert seen == len(b)
