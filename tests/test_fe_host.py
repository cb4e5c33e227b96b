"""The engine's device field arithmetic (firedancer_amd/csrc/
fd_ed25519_gpu_fe.h, whose functions are __host__ __device__) compiled for
the host and compared limb for limb with the reference's AVX field path
(oracle/_ref build) and the oracle restatement: fe_mul, fe_sqn (n=1,2)
over the operand ranges the verify path produces and past them (28-bit
limbs exercise the mod-2^32 operand pre-scales); the canonical encoding
and inversion used by the portable mode against the oracle's
fe_tobytes / field inverse.  Runs on the CPU: a kernel arithmetic change
is checked here before it ever reaches the GPU."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from conftest import P, ROOT

P25519 = 2**255 - 19


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    out = tmp_path_factory.mktemp("fehost") / "fehost.so"
    src = os.path.join(ROOT, "tests", "fe_host_harness.cpp")
    inc = ["-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(ROOT, "firedancer_amd", "csrc")]
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O2", "-std=c++17", "-fPIC", "-shared",
                    *inc, src, "-o", str(out)], check=True, capture_output=True)
    return ctypes.CDLL(str(out))


def rand_fe(rng, n, bits):
    return rng.integers(-(1 << (bits - 1)), 1 << (bits - 1), (n, 10), dtype=np.int64).astype(np.int32)


def value(f):
    """integer value of a radix-2^25.5 limb vector"""
    v, sh = 0, 0
    for i, x in enumerate(f):
        v += int(x) << sh
        sh += 25 if i & 1 else 26
    return v % P25519


@pytest.mark.parametrize("bits", [25, 26, 27, 28])
def test_mul_sqn_vs_reference(harness, ref, bits):
    rng = np.random.default_rng(bits)
    n = 4000
    F, G = rand_fe(rng, n, bits), rand_fe(rng, n, bits)
    H = np.zeros_like(F)
    harness.h_fe_mul(P(H), P(F), P(G), ctypes.c_ulong(n))
    for i in range(n):
        e = np.zeros(10, np.int32)
        ref.ref_fe_mul_avx(P(e), P(np.ascontiguousarray(F[i])), P(np.ascontiguousarray(G[i])))
        assert (H[i] == e).all(), (bits, i)
    # the latency kernel's product (independent column chains + the
    # reference carry chain on biased sums)
    H2 = np.zeros_like(F)
    harness.h_fe_mul_ilp(P(H2), P(F), P(G), ctypes.c_ulong(n))
    assert (H2 == H).all(), bits
    for nsq in (1, 2):
        harness.h_fe_sqn(P(H), P(F), nsq, ctypes.c_ulong(n))
        for i in range(n):
            e = np.zeros(10, np.int32)
            ref.ref_fe_sqn_avx(P(e), P(np.ascontiguousarray(F[i])), nsq)
            assert (H[i] == e).all(), (bits, nsq, i)


def test_carry_edges_vs_oracle(harness, oracle):
    """limbs at the carry rounding boundaries (+-2^24, +-2^25) and zero"""
    edges = np.array([0, 1, -1, 1 << 24, -(1 << 24), (1 << 24) - 1, 1 << 25, -(1 << 25), (1 << 25) - 1,
                      (1 << 26) - 1, -(1 << 26)], np.int32)
    rng = np.random.default_rng(9)
    F = rng.choice(edges, (3000, 10)).astype(np.int32)
    G = rng.choice(edges, (3000, 10)).astype(np.int32)
    H = np.zeros_like(F)
    harness.h_fe_mul(P(H), P(F), P(G), ctypes.c_ulong(len(F)))
    for i in range(len(F)):
        e = np.zeros(10, np.int32)
        oracle.oracle_fe_mul_avx(P(e), P(np.ascontiguousarray(F[i])), P(np.ascontiguousarray(G[i])))
        assert (H[i] == e).all(), i
    harness.h_fe_sqn(P(H), P(F), 2, ctypes.c_ulong(len(F)))
    for i in range(len(F)):
        e = np.zeros(10, np.int32)
        oracle.oracle_fe_sqn_avx(P(e), P(np.ascontiguousarray(F[i])), 2)
        assert (H[i] == e).all(), i


def test_tobytes_and_invert(harness, oracle):
    rng = np.random.default_rng(5)
    F = rand_fe(rng, 500, 26)
    F[0] = 0
    F[1] = np.array([-19, 0, 0, 0, 0, 0, 0, 0, 0, 1 << 25], np.int32)      # == 0 mod p, non-canonical
    W = np.zeros((len(F), 8), np.uint32)
    harness.h_fe_tobytes32(P(W), P(F), ctypes.c_ulong(len(F)))
    for i in range(len(F)):
        e = np.zeros(32, np.uint8)
        oracle.oracle_fe_tobytes(P(e), P(np.ascontiguousarray(F[i])))
        assert W[i].view(np.uint8).tobytes() == e.tobytes(), i
    I = np.zeros_like(F)
    harness.h_fe_invert(P(I), P(F), ctypes.c_ulong(len(F)))
    for i in range(2, len(F)):
        assert value(I[i]) * value(F[i]) % P25519 == 1
