"""Messages longer than the engine's staging blob.

The reference verifies a message of any length (fd_ed25519.h:96-101;
fd_sha512_append streams it, src/ballet/sha512/fd_sha512.c:282-349).  The
engine stages a batch's bytes in a pinned blob of max_blob bytes; a message
that does not fit is hashed on the device in blob-sized pieces with the
SHA-512 chaining state kept in HBM between launches (fd_k_sha512_stream),
then verified by the same prep (digest fed in), decompression and DSM code
as every batch.  Parity: codes equal the reference's own fd_ed25519_verify
(oracle/_ref/libfdref.so) on identical inputs -- valid and corrupted
signatures over 3 MB and 5 MB messages on an engine with a 1 MB blob, at
the short/long boundary, mixed with short messages; through the engine's
pointer-batch API and, in a child process whose default engine has a 1 MB
blob, through fd_ed25519_verify (4 threads), fd_ed25519_verify_batch and
fd_ed25519_verify_batch_single_msg."""
import ctypes
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import firedancer_amd as fa
from conftest import ROOT

MB = 1 << 20
BLOB = MB                       # engine staging blob: the long path starts at BLOB - 96 + 1
LIM = BLOB - 96


def _keypair(rng):
    L = fa.lib()
    priv = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    pub = ctypes.create_string_buffer(32)
    L.fd_ed25519_public_from_private(pub, priv, None)
    return priv, pub.raw


def _sign(msg, priv, pub):
    sig = ctypes.create_string_buffer(64)
    fa.lib().fd_ed25519_sign(sig, msg.ctypes.data if len(msg) else None, len(msg), pub, priv, None)
    return sig.raw


def _cases(seed):
    """(msg uint8 array, sig, pub, what) -- long, boundary and short"""
    rng = np.random.default_rng(seed)
    out = []
    for sz in (3 * MB, 5 * MB, LIM + 1, LIM, 1232 - 65, 0):
        m = rng.integers(0, 256, sz, dtype=np.uint8)
        priv, pub = _keypair(rng)
        sig = _sign(m, priv, pub)
        out.append((m, sig, pub, f"valid {sz}"))
        if sz >= 3 * MB:
            bad = m.copy()
            bad[-1] ^= 0x40                                 # last byte: in the final piece
            out.append((bad, sig, pub, f"msg flip end {sz}"))
            bad2 = m.copy()
            bad2[sz // 2] ^= 1                              # a middle piece
            out.append((bad2, sig, pub, f"msg flip mid {sz}"))
            r = bytearray(sig)
            r[5] ^= 2
            out.append((m, bytes(r), pub, f"R flip {sz}"))
            s = bytearray(sig)
            s[63] = 0xff                                    # S >= L: ERR_SIG before any hash
            out.append((m, bytes(s), pub, f"S>=L {sz}"))
            q1 = bytearray(sig)
            q1[63] = 0x10
            q1[50] |= 1                                     # the reference's early accept
            out.append((m, bytes(q1), pub, f"Q1 {sz}"))
            out.append((m, sig, bytes(32), f"small-order A {sz}"))
            out.append((m, sig, bytes(pub[:31]) + bytes([pub[31] ^ 0x80]), f"A sign flip {sz}"))
    return out


def _expected(ref, cases):
    return np.array([ref.ref_verify(m.ctypes.data if len(m) else None, len(m), s, p) for m, s, p, _ in cases], np.int32)


@pytest.mark.gpu
def test_long_messages_engine_batch_vs_reference(ref):
    cases = _cases(11)
    exp = _expected(ref, cases)
    assert (exp == 0).sum() >= 5 and (exp != 0).sum() >= 8
    eng = fa.Engine(0, 64, BLOB, depth=2)
    try:
        r, got = eng.verify_ptrs([c[0] for c in cases], [c[1] for c in cases], [c[2] for c in cases])
        bad = [(cases[i][3], int(got[i]), int(exp[i])) for i in np.nonzero(got != exp)[0]]
        assert not bad, bad
        first = exp[exp != 0]
        assert r == (int(first[0]) if len(first) else 0)
        # every mode runs the long path through its own checks: the strict
        # mode still accepts the valid ones and rejects the corrupted
        eng.mode = fa.MODE_STRICT
        r2, got2 = eng.verify_ptrs([c[0] for c in cases], [c[1] for c in cases], [c[2] for c in cases])
        for (m, s, p, what), g, e in zip(cases, got2, exp):
            if what.startswith("valid"):
                assert g == 0, what
            elif what.startswith(("msg", "R flip")):
                assert g != 0, what
    finally:
        eng.close()


@pytest.mark.gpu
def test_long_messages_reference_drop_ins_vs_reference(ref, tmp_path):
    cases = _cases(12)
    exp = _expected(ref, cases)
    rng = np.random.default_rng(13)
    shared = rng.integers(0, 256, 3 * MB + 17, dtype=np.uint8)
    ssig, spub = [], []
    for k in range(6):
        priv, pub = _keypair(rng)
        ssig.append(_sign(shared, priv, pub))
        spub.append(pub)
    s = bytearray(ssig[3])
    s[9] ^= 4
    ssig[3] = bytes(s)                                      # one corrupted signer
    sexp = np.array([ref.ref_verify(shared.ctypes.data, len(shared), a, b) for a, b in zip(ssig, spub)], np.int32)
    assert (sexp == 0).sum() == 5 and sexp[3] != 0
    npz = tmp_path / "cases.npz"
    np.savez(npz, n=len(cases), sig=np.array([np.frombuffer(c[1], np.uint8) for c in cases]),
             pub=np.array([np.frombuffer(c[2], np.uint8) for c in cases]), shared=shared,
             ssig=np.array([np.frombuffer(x, np.uint8) for x in ssig]), spub=np.array([np.frombuffer(x, np.uint8) for x in spub]),
             **{f"m{i}": c[0] for i, c in enumerate(cases)})
    out = tmp_path / "out.json"
    env = dict(os.environ, FD_ED25519_GPU_DEFAULT_BLOB=str(BLOB), PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "long_msg_child.py"), str(npz), str(out)],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    got = json.load(open(out))
    assert got["max_blob"] == BLOB
    names = [c[3] for c in cases]
    assert got["per"] == exp.tolist(), [(n, g, e) for n, g, e in zip(names, got["per"], exp.tolist()) if g != e]
    assert got["batch"] == exp.tolist()
    first = exp[exp != 0]
    assert got["batch_r"] == (int(first[0]) if len(first) else 0)
    assert got["single"] == sexp.tolist() and got["single_r"] == int(sexp[3])
