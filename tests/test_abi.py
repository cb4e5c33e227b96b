"""The C-ABI boundary: the product library loads and exports every
function include/*.h declares; without a gfx950 device it fails loudly
(no CPU fallback).  No compute call needs a GPU here."""
import ctypes
import glob
import os
import re

import numpy as np
import pytest

import firedancer_amd as fa
from conftest import ROOT, oracle_batch
from firedancer_amd import corpus


def declared_functions():
    names = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        txt = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        inline = set(re.findall(r"static\s+inline[^(]*?\b(fd_[a-z0-9_]+)\s*\(", txt, flags=re.S))
        for m in re.finditer(r"\b(fd_[a-z0-9_]+)\s*\(", txt):
            if m.group(1) not in inline:
                names.add(m.group(1))
    return sorted(names)


def test_header_declares_reference_surface():
    names = declared_functions()
    for must in ("fd_ed25519_verify", "fd_ed25519_strerror", "fd_ed25519_verify_batch",
                 "fd_ed25519_verify_batch_single_msg", "fd_ed25519_gpu_new", "fd_ed25519_gpu_submit",
                 "fd_ed25519_gpu_poll", "fd_ed25519_gpu_verify_dev"):
        assert must in names


def test_library_exports_every_declared_symbol():
    L = fa.lib()
    missing = [n for n in declared_functions() if not hasattr(L, n)]
    assert not missing, missing


def test_error_codes_match_reference():
    # fd_ed25519.h:11-14
    assert (fa.SUCCESS, fa.ERR_SIG, fa.ERR_PUBKEY, fa.ERR_MSG) == (0, -1, -2, -3)
    assert fa.strerror(0) == "success" and fa.strerror(-1) == "bad signature"
    assert fa.strerror(-2) == "bad public key" and fa.strerror(-3) == "bad message"
    assert fa.strerror(12345) == "unknown"


def test_no_gpu_fails_loudly():
    if fa.device_count() > 0:
        pytest.skip("a gfx950 device is present")
    assert fa.lib().fd_ed25519_gpu_new(0, 16, 4096) is None
    assert fa.last_error()
    r = fa.verify(b"abc", b"\0" * 64, b"\0" * 32)
    assert r == fa.ERR_GPU
    with pytest.raises(fa.EngineError):
        fa.Engine(0, 16, 4096)


def test_host_signer_matches_oracle_signer_and_verifies(oracle):
    b = corpus.simple(300, 77, seed=9)
    assert (oracle_batch(oracle, b) == 0).all()
    # the product signer and the oracle's signer agree byte for byte
    seeds = np.random.default_rng(9).integers(0, 256, (300, 32), dtype=np.uint8)
    sig, pub, data, off, sz = b.flat()
    pub2, sig2 = np.zeros_like(pub), np.zeros_like(sig)
    P = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    oracle.oracle_sign_batch(ctypes.c_uint64(300), P(seeds), P(data), P(off), P(sz), P(pub2), P(sig2), 4)
    assert (pub == pub2).all() and (sig == sig2).all()


def test_corpus_shapes():
    b = corpus.solana_txns(1000, seed=1)
    assert len(b) == 1000
    assert set(np.unique(b.desc["msg_sz"]).tolist()) <= {1167, 1103}
    a = corpus.adversarial(400, 128, seed=1)
    assert (a.label > 0).sum() == 40


def test_bounded_wait_selftest():
    """fd_event_wait's bounded poll (fd_ed25519_gpu_set_timeout) on a fake
    ticket, no device: a stuck ticket times out in about the timeout, a
    late one completes (the reference bounds its accelerator poll the
    same way, src/wiredancer/c/wd_f1.h:25)"""
    import time
    L = fa.lib()
    t0 = time.perf_counter()
    assert L.fd_ed25519_gpu_wait_selftest(30_000_000, -1) == 0          # never ready: 30 ms timeout
    dt = time.perf_counter() - t0
    assert 0.025 < dt < 1.0, dt
    assert L.fd_ed25519_gpu_wait_selftest(2_000_000_000, 40_000_000) == 1  # ready after 40 ms (past the spin)
    assert L.fd_ed25519_gpu_wait_selftest(2_000_000_000, 0) == 1
    assert L.fd_ed25519_gpu_wait_selftest(1_000_000, 500_000_000) == 0   # late: timed out first


def test_feeder_wait_keeps_arrays_until_final_state():
    """Feeder.wait: a wait that times out leaves the job queued
    or in flight on the feeder thread, so the blob, descriptors and out
    array it references must stay alive; they are released only once the
    job's state is final.  Driven through the real fd_ed25519_gpu_job_wait
    on a job no feeder ever completes (no device needed)."""
    f = fa.Feeder.__new__(fa.Feeder)
    f._h, f._keep = None, {}
    j = fa.Job()
    j.state = 0
    arrays = (np.zeros(8, np.uint8), np.zeros(1, fa.DESC_DTYPE), np.zeros(1, np.int32))
    f._keep[ctypes.addressof(j)] = arrays
    with pytest.raises(fa.EngineError):
        f.wait(j, 2_000_000)                  # 2 ms: times out, job still pending
    assert f._keep[ctypes.addressof(j)] is arrays
    j.state = 1                               # the feeder finished it
    f.wait(j, 2_000_000)
    assert ctypes.addressof(j) not in f._keep
    j2 = fa.Job()
    j2.state = fa.ERR_GPU                     # a failed job is final too
    f._keep[ctypes.addressof(j2)] = arrays
    with pytest.raises(fa.EngineError):
        f.wait(j2, 0)
    assert ctypes.addressof(j2) not in f._keep
