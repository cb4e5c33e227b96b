"""TEST INFRASTRUCTURE: helpers around tests/vt_live.cpp -- the verify tile
task run by its own loop and fed by a live producer over an mcache/dcache
link shaped like the reference's QUIC -> verify link (no flush, HALT only
at the end).  Used by tests/test_verify_tile_live.py, tests/test_sanitize.py
and tools/task_c5.py."""
import json
import os
import struct
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DIAG = ("IN_BACKP", "BACKP_CNT", "HA_FILT_CNT", "HA_FILT_SZ", "SV_FILT_CNT", "SV_FILT_SZ",
        "PUB_CNT", "PUB_SZ", "BAD_CNT", "SIG_CNT", "BATCH_CNT", "RING_FULL_CNT", "OVRN_CNT", "AGE_CNT")


def quiet_cpus(n, device=0, sample_s=0.3, pairs=True):
    """n quiet CPUs of the GPU's NUMA node as "c0,c1,..." (firedancer_amd.
    quiet_cpus: producer k and tile k share a last-level cache), or None"""
    import firedancer_amd as fa
    pick = fa.quiet_cpus(n, device, sample_s, pairs)
    return ",".join(str(x) for x in pick) if pick else None


def write_frags(path, frags):
    """the corpus file: u32 n, then n x (u32 sz, bytes)"""
    with open(path, "wb") as f:
        f.write(struct.pack("<I", len(frags)))
        for fr in frags:
            f.write(struct.pack("<I", len(fr)) + bytes(fr))


def write_expect(path, flags):
    """per corpus entry: 1 if the reference tile publishes it"""
    np.asarray(flags, np.uint8).tofile(path)


def read_pubout(path):
    """(seq, tspub - tsorig ns) of every publish, in publish order"""
    a = np.fromfile(path, np.uint64)
    return a.reshape(-1, 2)


def run(exe, frags_path, timeout=300, env=None, **kw):
    """run the harness; returns its JSON line as a dict (+ rc, stderr tail)"""
    args = [exe, frags_path] + [f"{k}={v}" for k, v in kw.items()]
    try:
        r = subprocess.run(args, capture_output=True, text=True, timeout=timeout, env=env)
    except subprocess.TimeoutExpired as e:      # killed at the limit: say where it was
        def txt(x):
            return x.decode(errors="replace") if isinstance(x, bytes) else (x or "")
        raise AssertionError(f"harness timed out after {timeout} s: {args[2:]}\nstdout: {txt(e.stdout)[-2000:]}"
                             f"\nstderr: {txt(e.stderr)[-4000:]}") from None
    lines = [x for x in r.stdout.strip().splitlines() if x.startswith("{")]
    assert lines, (r.returncode, r.stdout[-2000:], r.stderr[-3000:])
    d = json.loads(lines[-1])
    d["rc"] = r.returncode
    d["stderr"] = r.stderr[-3000:]
    if isinstance(d.get("diag"), list):
        d["diag"] = dict(zip(DIAG, d["diag"]))
    return d


def expected_cyclic(frags, ref, oracle_batch):
    """per-entry expectation for a corpus cycled through the tile: the
    reference's per-frag semantics (fd_frank_verify_synth_load.c:360-410)
    with every entry distinct (no HA duplicate across a cycle: the
    tcache's 16 tags never span a repeat when len(frags) > 16)"""
    from firedancer_amd import corpus, txn
    assert len(frags) > 16
    tags = set()
    blob, descs, owners, ok_parse = [], [], [], []
    off = 0
    for i, f in enumerate(frags):
        psz = int.from_bytes(f[-2:], "little")
        t = txn.parse(f[:psz]) if psz <= len(f) - 2 else None
        if t is None or psz > txn.TXN_MTU:
            ok_parse.append(False)
            continue
        tag = int.from_bytes(f[t["signature_off"]:t["signature_off"] + 8], "little")
        assert tag not in tags and tag != 0, "corpus entries must be distinct"
        tags.add(tag)
        d = txn.descs_for(f[:psz], off)
        blob.append(f)
        descs.append(d)
        owners += [i] * len(d)
        off += len(f)
        ok_parse.append(True)
    bb = corpus.Batch(np.frombuffer(b"".join(blob) + b"\0" * 64, np.uint8).copy(), np.concatenate(descs))
    codes = oracle_batch(ref, bb)
    ok = np.array(ok_parse, bool)
    np.logical_and.at(ok, np.array(owners), codes == 0)
    return ok


def expected_cheap(frags, ref):
    """expected_for (tests/test_verify_tile.py) with the fake engine's cheap
    codes (tests/sanitize/fake_engine.cpp: a signature whose first byte is
    odd fails): the reference tile's tcache and parse decisions, a stand-in
    verify -- for sanitizer runs whose point is the host logic, not the
    arithmetic.  -> published frags in order, counters"""
    from firedancer_amd import txn
    from test_verify_tile import _ref_tc
    r = _ref_tc(ref, 16, 64)
    pub, exp = [], dict(HA_FILT_CNT=0, HA_FILT_SZ=0, SV_FILT_CNT=0, SV_FILT_SZ=0, BAD_CNT=0)
    for f in frags:
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
        so, n = t["signature_off"], t["signature_cnt"]
        if all(f[so + 64 * k] % 2 == 0 for k in range(n)):
            pub.append(f)
        else:
            exp["SV_FILT_CNT"] += 1
            exp["SV_FILT_SZ"] += len(f)
    ref.ref_tcache_delete(r)
    return pub, exp
