"""The committed C5 record (profiles/r05_tile_c5_60s.jsonl, tools/bench_tile.py
--check-window on the GPU box) held against the reference on the CPU:
the frag set is regenerated from the record's seed, its first W frags run
through the reference's per-frag semantics
(/root/reference/src/app/frank/load/fd_frank_verify_synth_load.c:360-410:
the tcache of src/tango/tcache/fd_tcache.h and fd_ed25519_verify, both
from the oracle/_ref build, via tests/test_verify_tile.py's expected_for),
and the record's published stream (ordered frag indices, as a sha256) and
counters must be exactly the reference's."""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import ROOT

RECORD = os.path.join(ROOT, "profiles", "r05_tile_c5_60s.jsonl")


def _record():
    if not os.path.exists(RECORD):
        pytest.skip("no C5 record yet (tools/bench_tile.py --check-window on the GPU box)")
    rows = [json.loads(x) for x in open(RECORD) if x.strip().startswith("{")]
    rows = [r for r in rows if r.get("check_window")]
    assert rows, "no record with a check window"
    return rows[-1]


def test_c5_record_window_equals_reference(ref):
    from firedancer_amd import corpus, txn
    from test_verify_tile import _ref_tc
    rec = _record()
    chk = rec["check_window"]
    assert rec["seconds"] >= 60 and rec["latency_tsorig_to_tspub"]
    b = corpus.solana_txns(chk["sigs"], seed=chk["seed"], sig_dist=[1 / 12] * 12, nthreads=min(16, os.cpu_count() or 8))
    starts = sorted({int(d["sig_off"]) // corpus.TXN_MTU * corpus.TXN_MTU for d in b.desc})
    frags = [txn.frag(bytes(b.blob[s:s + corpus.TXN_MTU])) for s in starts[:chk["frags"]]]
    if chk.get("edits") == "corpus.c5_check_edits":
        frags = corpus.c5_check_edits(frags)
    # the reference's per-frag semantics, keeping each published frag's index
    r = _ref_tc(ref, 16, 64)
    cand, descs, owners, blob, off = [], [], [], [], 0
    ha = bad = 0
    for i, f in enumerate(frags):
        psz = int.from_bytes(f[-2:], "little")
        t = txn.parse(f[:psz]) if psz <= len(f) - 2 else None
        if t is None or psz > txn.TXN_MTU:
            bad += 1
            continue
        tag = int.from_bytes(f[t["signature_off"]:t["signature_off"] + 8], "little")
        if ref.ref_tcache_insert(r, tag):
            ha += 1
            continue
        d = txn.descs_for(f[:psz], off)
        blob.append(f)
        descs.append(d)
        owners += [len(cand)] * len(d)
        cand.append(i)
        off += len(f)
    ref.ref_tcache_delete(r)
    from conftest import oracle_batch
    bb = corpus.Batch(np.frombuffer(b"".join(blob) + b"\0" * 64, np.uint8).copy(), np.concatenate(descs))
    codes = oracle_batch(ref, bb)
    ok = np.ones(len(cand), bool)
    np.logical_and.at(ok, np.array(owners), codes == 0)
    pub = np.array([c for c, g in zip(cand, ok) if g], np.uint64)
    assert len(pub) == chk["published"]
    assert hashlib.sha256(pub.tobytes()).hexdigest() == chk["pub_ctl_sha256"]
    if chk.get("edits"):      # the edits reach every branch of the per-frag semantics
        assert ha > 0 and bad > 0 and (~ok).sum() > 0
    d = chk["diag"]
    assert d["PUB_CNT"] == len(pub) and d["SV_FILT_CNT"] == int((~ok).sum())
    assert d["HA_FILT_CNT"] == ha and d["BAD_CNT"] == bad and d["SIG_CNT"] == len(codes)
