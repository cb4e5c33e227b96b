"""The quad DSM's step (fd_quad_body,
firedancer_amd/csrc/fd_ed25519_gpu_kernels.hip) restated on the host with
the quad's four lanes as an array (tests/fe_host_harness.cpp h_quad_dsm:
the same fd_q3_entry decode table, raw products fd_fe_mul_raw and op
stream fd_recode as the kernel) and held limb for limb against the
reference's double-scalar multiplication, fd_ed25519_ge_double_scalarmult_
vartime (/root/reference/src/ballet/ed25519/avx/fd_ed25519_ge.c:405-527,
oracle/_ref build), whose p2 limbs are what the Q2 compare reads.  Also
pins the two facts the layout leans on: the commuted product t3 t0 equals
the reference's t0 t3 over every limb size the DSM produces (no 2f / 19g
pre-scale wraps below 2^26.75), and the biased product minus its biases is
fd_fe_mul."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from conftest import P, ROOT

FD_OPS_MAX = 512
L_ORDER = 2**252 + 27742317777372353535851937790883648493


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    out = tmp_path_factory.mktemp("quadmodel") / "fehost.so"
    src = os.path.join(ROOT, "tests", "fe_host_harness.cpp")
    inc = ["-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(ROOT, "firedancer_amd", "csrc")]
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O2", "-std=c++17", "-fPIC", "-shared",
                    *inc, src, "-o", str(out)], check=True, capture_output=True)
    L = ctypes.CDLL(str(out))
    L.h_quad_dsm.restype = ctypes.c_int
    return L


def points(oracle, ref, n, seed):
    """n decompressed public keys (p3 limbs X, Y, Z, T) of random seeds"""
    rng = np.random.default_rng(seed)
    out = []
    while len(out) < n:
        priv = rng.integers(0, 256, 32, dtype=np.uint8)
        pub = np.zeros(32, np.uint8)
        oracle.oracle_public_from_private(P(pub), P(priv))
        a = np.zeros(40, np.int32)
        b = np.zeros(40, np.int32)
        if ref.ref_ge_frombytes_2(P(a), P(pub), P(b), P(pub)) == 0:
            out.append(a)
    return out


def scalar(rng, top):
    v = int.from_bytes(rng.integers(0, 256, 32, dtype=np.uint8).tobytes(), "little") % top
    return np.frombuffer(v.to_bytes(32, "little"), np.uint8).copy()


def run_case(harness, ref, A, a, b):
    ops = np.zeros(FD_OPS_MAX, np.uint8)
    start = np.zeros(1, np.int32)
    harness.h_recode(P(ops), P(start), P(b), P(a), ctypes.c_ulong(1))
    got = np.zeros(30, np.int32)
    mx = np.zeros(1, np.int32)
    harness.h_quad_dsm(P(got), P(A), P(ops), int(start[0]), P(mx))
    exp = np.zeros(30, np.int32)
    ref.ref_ge_dsm(P(exp), P(a), P(A), P(b))
    return got, exp, int(mx[0])


def test_quad_step_layout_vs_reference_dsm(harness, oracle, ref):
    rng = np.random.default_rng(2025)
    pts = points(oracle, ref, 24, 7)
    worst = 0
    for i in range(240):
        A = pts[i % len(pts)]
        a = scalar(rng, L_ORDER)
        b = scalar(rng, L_ORDER)
        got, exp, mx = run_case(harness, ref, A, a, b)
        assert (got == exp).all(), i
        worst = max(worst, mx)
    # every product operand of the loop stays where 19 x (the pre-scale of
    # the commuted operand) cannot wrap int32
    assert worst * 19 < 2**31, worst


def test_quad_step_layout_edge_scalars(harness, oracle, ref):
    """zero, one, small and top-of-range scalars (short and long op streams,
    all-doubling tails, digits of both signs from both tables)"""
    pts = points(oracle, ref, 4, 11)
    vals = [0, 1, 2, 15, 16, 17, 31, 2**252, L_ORDER - 1, 2**253 - 1, int("5" * 75) % L_ORDER]
    for i, x in enumerate(vals):
        for j, y in enumerate(vals):
            a = np.frombuffer(x.to_bytes(32, "little"), np.uint8).copy()
            b = np.frombuffer(y.to_bytes(32, "little"), np.uint8).copy()
            got, exp, _ = run_case(harness, ref, pts[(i + j) % 4], a, b)
            assert (got == exp).all(), (x, y)


def test_commuted_product_in_range(harness, ref):
    """g f == the reference's f g while |limbs| < 2^31 / 19 (the DSM's
    operands stay below 3 * 2^25 + 2^12); at 28-bit limbs the wrapped
    pre-scales make the order matter, which is why only that range may
    commute"""
    rng = np.random.default_rng(4)
    n = 4000
    lim = (2**31 - 1) // 19
    F = rng.integers(-lim, lim + 1, (n, 10), dtype=np.int64).astype(np.int32)
    G = rng.integers(-lim, lim + 1, (n, 10), dtype=np.int64).astype(np.int32)
    H = np.zeros_like(F)
    harness.h_fe_mul_swapped(P(H), P(F), P(G), ctypes.c_ulong(n))
    for i in range(n):
        e = np.zeros(10, np.int32)
        ref.ref_fe_mul_avx(P(e), P(np.ascontiguousarray(F[i])), P(np.ascontiguousarray(G[i])))
        assert (H[i] == e).all(), i
    F = rng.integers(-(1 << 27), 1 << 27, (200, 10), dtype=np.int64).astype(np.int32)
    G = rng.integers(-(1 << 27), 1 << 27, (200, 10), dtype=np.int64).astype(np.int32)
    H = np.zeros_like(F)
    harness.h_fe_mul_swapped(P(H), P(F), P(G), ctypes.c_ulong(200))
    diff = 0
    for i in range(200):
        e = np.zeros(10, np.int32)
        ref.ref_fe_mul_avx(P(e), P(np.ascontiguousarray(F[i])), P(np.ascontiguousarray(G[i])))
        diff += int(not (H[i] == e).all())
    assert diff > 0


def test_biased_product(harness):
    rng = np.random.default_rng(8)
    F = rng.integers(-(1 << 27), 1 << 27, (3000, 10), dtype=np.int64).astype(np.int32)
    G = rng.integers(-(1 << 27), 1 << 27, (3000, 10), dtype=np.int64).astype(np.int32)
    H1 = np.zeros_like(F)
    H2 = np.zeros_like(F)
    harness.h_fe_mul(P(H1), P(F), P(G), ctypes.c_ulong(len(F)))
    harness.h_fe_mul_b(P(H2), P(F), P(G), ctypes.c_ulong(len(F)))
    assert (H1 == H2).all()


def test_op_streams_start_inside_the_lds_rows(harness):
    """The quad DSM keeps op rows from t = 144 on (FD_QOPS_BASE): a stream
    of two scalars below 2^253 holds at most 2 x 51 width-5 digits, so it
    starts at 512 - 256 - 102 = 154 or later.  Checked on random scalars and
    on the densest patterns (every bit set, alternating bits, a digit every
    fifth bit) at the top of the range."""
    rng = np.random.default_rng(31)
    dense = [2**253 - 1, int("01" * 126, 2), int("10" * 126, 2), sum(1 << (5 * i) for i in range(51)),
             sum(1 << (5 * i + 4) for i in range(50)), L_ORDER - 1, int("1" * 252 + "0", 2)]
    cases = [(a, b) for a in dense for b in dense]
    cases += [(int(rng.integers(0, 2**63)) << 189 | int(rng.integers(0, 2**63)), int(rng.integers(0, 2**62)) << 190) for _ in range(500)]
    low = FD_OPS_MAX
    for a, b in cases:
        a %= 2**253
        b %= 2**253
        ops = np.zeros(FD_OPS_MAX, np.uint8)
        start = np.zeros(1, np.int32)
        A = np.frombuffer(a.to_bytes(32, "little"), np.uint8).copy()
        B = np.frombuffer(b.to_bytes(32, "little"), np.uint8).copy()
        harness.h_recode(P(ops), P(start), P(B), P(A), ctypes.c_ulong(1))
        low = min(low, int(start[0]))
        assert int(start[0]) >= 154, (hex(a), hex(b), int(start[0]))
    assert low < 200
