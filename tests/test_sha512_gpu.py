"""SHA-512 batch API GPU backend (include/fd_sha512_gpu.h; SURVEY.md
section 8f row 3).  Digests are checked against NIST CAVP vectors and the
reference's own vectors (tests/golden/sha512_vectors.json) and against
the reference's fd_sha512 / fd_sha384 compiled in place (oracle/_ref) on
random messages at every padding boundary."""
import ctypes

import numpy as np
import pytest

import firedancer_amd as fa
from conftest import ROOT  # noqa: F401
from test_oracle import shavec  # noqa: F401  (fixture)


def ref_hash(ref, msg, is384=False):
    fn = ref.ref_sha384 if is384 else ref.ref_sha512
    fn.argtypes = [ctypes.c_char_p, ctypes.c_ulong, ctypes.c_void_p]
    out = ctypes.create_string_buffer(64)
    fn(bytes(msg), len(msg), out)
    return out.raw[:48 if is384 else 64]


def boundary_msgs(rng):
    sizes = sorted({s + d for s in (0, 111, 112, 128, 239, 240, 256, 1167, 1232) for d in (-1, 0, 1) if s + d >= 0})
    sizes += [int(x) for x in rng.integers(0, 4000, 200)]
    return [rng.integers(0, 256, s, dtype=np.uint8).tobytes() for s in sizes]


def test_batch_api_exported():
    L = fa.lib()
    for n in ("fd_sha512_gpu_batch_new", "fd_sha512_gpu_batch_add", "fd_sha512_gpu_batch_fini",
              "fd_sha512_gpu_batch_abort", "fd_ed25519_gpu_sha512_packed"):
        assert hasattr(L, n)
    if fa.device_count() == 0:
        assert L.fd_sha512_gpu_batch_new(None, 0) is None      # no device: no CPU fallback


@pytest.mark.gpu
def test_cavp_and_fd_vectors(engine, shavec):
    for key in ("cavp_short", "cavp_long", "fd_test_vector"):
        vs = shavec[key]
        got = engine.sha512([bytes.fromhex(v["msg"]) for v in vs])
        assert [g.hex() for g in got] == [v["md"] for v in vs], key


@pytest.mark.gpu
@pytest.mark.parametrize("is384", [False, True])
def test_random_vs_reference(engine, ref, is384):
    msgs = boundary_msgs(np.random.default_rng(3 + is384))
    got = engine.sha512(msgs, is384=is384)
    assert got == [ref_hash(ref, m, is384) for m in msgs]


@pytest.mark.gpu
def test_batch_add_fini_abort(ref):
    L = fa.lib()
    b = L.fd_sha512_gpu_batch_new(None, 0)
    assert b
    rng = np.random.default_rng(8)
    msgs = [rng.integers(0, 256, int(rng.integers(0, 1500)), dtype=np.uint8).tobytes() for _ in range(5000)]
    bufs = [ctypes.create_string_buffer(m, max(1, len(m))) for m in msgs]
    outs = [ctypes.create_string_buffer(64) for _ in msgs]
    L.fd_sha512_gpu_batch_init(b)
    for m, buf, o in zip(msgs, bufs, outs):
        L.fd_sha512_gpu_batch_add(b, buf, len(m), o)
    assert L.fd_sha512_gpu_batch_fini(b) == b
    assert all(o.raw == ref_hash(ref, m) for m, o in zip(msgs, outs))
    # abort drops the queue: nothing written
    o = ctypes.create_string_buffer(b"\xaa" * 64, 64)
    L.fd_sha512_gpu_batch_add(L.fd_sha512_gpu_batch_init(b), bufs[0], len(msgs[0]), o)
    L.fd_sha512_gpu_batch_abort(b)
    assert L.fd_sha512_gpu_batch_fini(b) == b and o.raw == b"\xaa" * 64
    L.fd_sha512_gpu_batch_delete(b)
