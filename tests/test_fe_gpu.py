"""The engine's field products as DEVICE code (fd_k_debug_fe: the same
fd_ed25519_gpu_fe.h functions the kernels are built from, compiled for
gfx950 with their value barriers) compared limb for limb with the
reference's AVX field ops (oracle/_ref build: FE_AVX_INL_MUL and SQN,
src/ballet/ed25519/avx/fd_ed25519_fe_avx_inl.h:484-677), over the operand
ranges the verify path produces and past them (28-bit limbs exercise the
mod-2^32 operand pre-scales).  tests/test_fe_host.py checks the host
compile of the same functions; end-to-end parity checks them only through
verdicts.  Row a8 of SURVEY.md section 8."""
import numpy as np
import pytest

from conftest import P

pytestmark = pytest.mark.gpu

N = 4096


def rand_fe(rng, n, bits):
    return rng.integers(-(1 << (bits - 1)), 1 << (bits - 1), (n, 10), dtype=np.int64).astype(np.int32)


def ref_mul(ref, F, G):
    out = np.zeros_like(F)
    for i in range(len(F)):
        e = np.zeros(10, np.int32)
        ref.ref_fe_mul_avx(P(e), P(np.ascontiguousarray(F[i])), P(np.ascontiguousarray(G[i])))
        out[i] = e
    return out


def ref_sqn(ref, F, n):
    out = np.zeros_like(F)
    for i in range(len(F)):
        e = np.zeros(10, np.int32)
        ref.ref_fe_sqn_avx(P(e), P(np.ascontiguousarray(F[i])), n)
        out[i] = e
    return out


@pytest.mark.parametrize("bits", [25, 26, 27, 28])
def test_device_field_products_vs_reference(engine, ref, bits):
    rng = np.random.default_rng(100 + bits)
    F, G = rand_fe(rng, N, bits), rand_fe(rng, N, bits)
    fg, gf, ff = ref_mul(ref, F, G), ref_mul(ref, G, F), ref_mul(ref, F, F)
    f2, g2x2 = ref_sqn(ref, F, 1), ref_sqn(ref, G, 2)
    f2x2 = ref_sqn(ref, F, 2)
    H = {op: engine.debug_fe(op, F, G) for op in range(8)}
    assert (H[0][0] == fg).all(), "fd_fe_mul"
    assert (H[1][0] == f2).all(), "fd_fe_sqn n=1"
    assert (H[2][0] == f2x2).all(), "fd_fe_sqn n=2"
    assert (H[3][0] == fg).all(), "fd_fe_mul_ilp"
    assert (H[4][0] == fg).all() and (H[4][1] == gf).all(), "fd_fe_mul2"
    assert (H[5][0] == fg).all() and (H[5][1] == gf).all() and (H[5][2] == ff).all(), "fd_fe_chain3"
    assert (H[6][0] == f2).all() and (H[6][1] == g2x2).all(), "fd_fe_sqn2"
    bad = np.nonzero((H[7][0] != fg).any(axis=1))[0]
    assert len(bad) == 0, ("fd_o_mul (oct DSM half product)", bad[:8], H[7][0][bad[:2]], fg[bad[:2]])


def test_device_field_products_args(engine):
    import firedancer_amd as fa
    with pytest.raises(fa.EngineError):
        engine.debug_fe(8, np.zeros((1, 10), np.int32), np.zeros((1, 10), np.int32))
    assert engine.debug_fe(0, np.zeros((0, 10), np.int32), np.zeros((0, 10), np.int32)).shape == (3, 0, 10)
