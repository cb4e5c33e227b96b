"""The eight-lane DSM's split product (fd_o_mul in
firedancer_amd/csrc/fd_ed25519_gpu_kernels.hip) restated lane by lane on
the host: each half forms five column sums with g rotated by five limbs in
the h = 1 half, the per-lane 2f / 19g rules, and the reference's 12-step
carry chain split over the halves (A: c4 into limb 5; B-E in both halves
at once; F: c4' and 19 c9 across; G: c0').  Checked limb for limb against
the reference's AVX MUL (oracle/_ref: FE_AVX_INL_MUL,
src/ballet/ed25519/avx/fd_ed25519_fe_avx_inl.h:484-590), including 28-bit
limbs where the 32-bit pre-scales wrap.  The device code itself is checked
the same way on the GPU (tests/test_fe_gpu.py, debug op 7)."""
import numpy as np
import pytest

from conftest import P

M64 = (1 << 64) - 1


def s32(x):
    x &= 0xffffffff
    return x - (1 << 32) if x >> 31 else x


def s64(x):
    x &= M64
    return x - (1 << 64) if x >> 63 else x


def u32(x):
    return x & 0xffffffff


def ash(x, w):
    return s64(x) >> w


def oct_mul(f, g):
    """both halves of fd_o_mul in lockstep; returns limbs 0-9"""
    own_f = [f[0:5], f[5:10]]
    own_g = [g[0:5], g[5:10]]
    st = []
    for h in (0, 1):
        F = own_f[0] + own_f[1]                          # natural order (fd_o_both)
        G = own_g[h] + own_g[1 - h]                      # [own, partner]
        FA = [s32(F[i] << (1 - h)) if i & 1 else None for i in range(10)]
        FB = [s32(F[i] << h) if i & 1 else None for i in range(10)]
        G19 = [0] + [s32(19 * G[j]) for j in range(1, 5)] + [s32((1 if h else 19) * G[j]) for j in range(5, 10)]
        wE, wO = (25, 26) if h else (26, 25)
        bE, bO = (1 << 24, 1 << 25) if h else (1 << 25, 1 << 24)
        S = [bE, bO, bE, bO, bE]
        for jp in range(10):
            for j in range(5):
                i = (j - jp + 10) % 10
                fo = (FA[i] if jp & 1 else FB[i]) if i & 1 else F[i]
                go = G[jp] if jp <= j else G19[jp]
                S[j] = s64(S[j] + fo * go)
        st.append({"S": S, "wE": wE, "wO": wO, "bE": bE, "bO": bO})
    # A: h = 0's first carry of limb 4 into limb 5
    c4 = ash(st[0]["S"][4], 26)
    st[0]["S"][4] = u32(st[0]["S"][4]) & ((1 << 26) - 1)
    st[1]["S"][0] = s64(st[1]["S"][0] + c4)
    # B-E: 0->1 .. 3->4 | 5->6 .. 8->9
    for x in st:
        S = x["S"]
        for j in range(4):
            w = x["wE"] if j % 2 == 0 else x["wO"]
            c = ash(S[j], w)
            S[j] = u32(S[j]) & ((1 << w) - 1)
            S[j + 1] = s64(S[j + 1] + c)
    # F: c4' into limb 5, 19 c9 into limb 0
    cy = []
    for x in st:
        S = x["S"]
        cy.append(ash(S[4], x["wE"]))
        S[4] = u32(S[4]) & ((1 << x["wE"]) - 1)
    st[0]["S"][0] = s64(st[0]["S"][0] + 19 * cy[1])
    st[1]["S"][0] = s64(st[1]["S"][0] + cy[0])
    # G: c0'
    S = st[0]["S"]
    c = ash(S[0], 26)
    S[0] = u32(S[0]) & ((1 << 26) - 1)
    S[1] = s64(S[1] + c)
    out = []
    for x in st:
        out += [s32(u32(x["S"][j]) - (x["bE"] if j % 2 == 0 else x["bO"])) for j in range(5)]
    return out


@pytest.mark.parametrize("bits", [25, 26, 27, 28])
def test_oct_split_product_equals_reference_mul(ref, bits):
    rng = np.random.default_rng(700 + bits)
    for _ in range(400):
        f = rng.integers(-(1 << (bits - 1)), 1 << (bits - 1), 10).astype(np.int32)
        g = rng.integers(-(1 << (bits - 1)), 1 << (bits - 1), 10).astype(np.int32)
        e = np.zeros(10, np.int32)
        ref.ref_fe_mul_avx(P(e), P(f), P(g))
        assert oct_mul([int(x) for x in f], [int(x) for x in g]) == [int(x) for x in e], (f, g)
