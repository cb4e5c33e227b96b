"""Shared fixtures.  GPU tests are marked @pytest.mark.gpu; everything
else runs on CPU.  The oracle (oracle/liboracle.so, and the reference
build oracle/_ref/libfdref.so when present) is test infrastructure: it is
the checker here, never the thing under test."""
import ctypes
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device")


def pytest_collection_modifyitems(session, config, items):
    """the live-producer latency tests (tests/test_verify_tile_live.py) run
    first, while this process holds no engine: each engine keeps CU-masked
    streams, and on AMD every such stream owns a hardware queue, so engines
    of earlier tests alive in this process push the GPU's scheduler into
    queue oversubscription, which time-slices the harness's queues in
    milliseconds -- a validator gives the GPU to its verify tiles alone"""
    first = [it for it in items if "test_verify_tile_live" in it.nodeid]
    if first:
        items[:] = first + [it for it in items if "test_verify_tile_live" not in it.nodeid]


def P(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _load_oracle():
    path = os.path.join(ROOT, "oracle", "liboracle.so")
    if not os.path.exists(path):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "oracle"], check=True, capture_output=True)
    L = ctypes.CDLL(path)
    L.oracle_verify.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]
    L.oracle_verify.restype = ctypes.c_int
    return L


@pytest.fixture(scope="session")
def oracle():
    return _load_oracle()


@pytest.fixture(scope="session")
def ref():
    path = os.path.join(ROOT, "oracle", "_ref", "libfdref.so")
    if not os.path.exists(path):
        if os.path.isdir("/root/reference"):
            subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "ref"], check=True, capture_output=True)
        else:
            # the reference build travels with the tree (built .so files are
            # shipped to the GPU box); a parity test never silently weakens
            pytest.fail(f"{path} missing: build it in the container with make -C oracle ref")
    L = ctypes.CDLL(path)
    L.ref_verify.argtypes = [ctypes.c_void_p, ctypes.c_ulong, ctypes.c_void_p, ctypes.c_void_p]
    L.ref_verify.restype = ctypes.c_int
    return L


def oracle_batch(L, b, threads=None):
    """Per-signature codes of a corpus.Batch from a checker library."""
    sig, pub, data, off, sz = b.flat()
    out = np.zeros(len(b), np.int32)
    th = threads or min(16, os.cpu_count() or 8)
    fn = L.oracle_verify_batch if hasattr(L, "oracle_verify_batch") else L.ref_verify_batch
    fn(ctypes.c_uint64(len(b)), P(sig), P(pub), P(data), P(off), P(sz), P(out), th)
    return out


def load_corpus(name):
    from firedancer_amd.corpus import Batch
    z = np.load(os.path.join(GOLDEN, f"corpus_{name}.npz"))
    return Batch(z["blob"], z["desc"], z["label"]), z["expected"]


def ed_vectors():
    return json.load(open(os.path.join(GOLDEN, "ed25519_vectors.json")))


def malleability():
    out = []
    for kind, ok in (("pass", True), ("fail", False)):
        raw = open(os.path.join(GOLDEN, f"malleability_should_{kind}.bin"), "rb").read()
        for i in range(len(raw) // 96):
            out.append((raw[96 * i:96 * i + 64], raw[96 * i + 64:96 * i + 96], ok))
    return out


@pytest.fixture(scope="session")
def engine():
    import firedancer_amd as fa
    if fa.device_count() < 1:
        pytest.fail("no gfx950 device visible to a -m gpu test")
    e = fa.Engine(0, 1 << 18, 1 << 28)
    yield e
    e.close()
