"""Wire parsing of the reference's txn fixtures (src/ballet/txn/fixtures)
and of the synthetic Solana-MTU corpus; every signature of the fixtures
verifies under the oracle (all 6 are valid)."""
import os

import numpy as np

from conftest import GOLDEN, oracle_batch
from firedancer_amd import corpus, txn


def fixtures():
    return [open(os.path.join(GOLDEN, f"transaction{i}.bin"), "rb").read() for i in (1, 2, 3)]


def test_parse_fixtures():
    t = [txn.parse(p) for p in fixtures()]
    assert [x["sig_cnt"] for x in t] == [4, 1, 1]
    assert [x["version"] for x in t] == [-1, 0, -1]


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
    assert txn.parse(p * 2) is None                  # > MTU


def test_synthetic_txns_parse():
    b = corpus.solana_txns(64, seed=3)
    bases = sorted({int(d["msg_off"]) - 1 - 64 * ((int(d["msg_sz"]) < 1167) + 1) for d in b.desc})
    for base in bases:
        t = txn.parse(bytes(b.blob[base:base + corpus.TXN_MTU]))
        assert t is not None and t["msg_off"] == 1 + 64 * t["sig_cnt"]
