"""The DSM op-stream recoder (firedancer_amd/csrc/fd_ed25519_gpu_wnaf.h,
__host__ __device__) compiled for the host and compared byte for byte
with the op stream built from the oracle's fd_ed25519_ge_slide
restatement (avx/fd_ed25519_ge.c:378-400) in the reference's DSM order
(avx/fd_ed25519_ge.c:490-523: per bit from 255 down, D, k's add, S's
add), over random scalars below 2^253 and edge scalars (0, 1, L-1,
2^252, long zero runs, dense ones).  CPU only."""
import ctypes

import numpy as np
import pytest

from conftest import P
from test_fe_host import harness  # noqa: F401  (module fixture)

FD_OPS_MAX = 512
L = 2**252 + 27742317777372353535851937790883648493


def expected_stream(oracle, s, k):
    ds = np.zeros(256, np.int8)
    dk = np.zeros(256, np.int8)
    oracle.oracle_ge_slide(P(ds), s.to_bytes(32, "little"))
    oracle.oracle_ge_slide(P(dk), k.to_bytes(32, "little"))
    seq = []
    for b in range(255, -1, -1):
        seq.append(0)
        for t, d in ((0, int(dk[b])), (1, int(ds[b]))):
            if d:
                seq.append(0x80 | (t << 6) | ((d < 0) << 5) | (abs(d) >> 1))
    out = np.zeros(FD_OPS_MAX, np.uint8)
    out[FD_OPS_MAX - len(seq):] = seq
    return out, FD_OPS_MAX - len(seq)


def edge_scalars():
    return [0, 1, 2, 15, 16, 17, 31, 32, L - 1, L - 2, 2**252, 2**252 - 1, 2**200, 2**64, 2**32 + 1,
            (2**253 - 1) // 3, 2**253 - 1 - 2**130, int("10000" * 50, 2), int("11111" * 50, 2),
            # a negative digit whose +2^5 carries out of the low word (and on
            # through all-ones words): the recoder's rare carry branch
            2**32 - 15, 2**64 - 15, 2**96 - 15, 2**224 - 15, (2**252 - 1) ^ 0x0e]


def test_recode_vs_oracle_slide(harness, oracle):  # noqa: F811
    rng = np.random.default_rng(11)
    ed = edge_scalars()
    pairs = [(a, b) for a in ed for b in ed[:6]] + [(int.from_bytes(rng.bytes(32), "little") % 2**253,
                                                      int.from_bytes(rng.bytes(32), "little") % L) for _ in range(1500)]
    n = len(pairs)
    S = np.frombuffer(b"".join(s.to_bytes(32, "little") for s, _ in pairs), np.uint8).copy()
    K = np.frombuffer(b"".join(k.to_bytes(32, "little") for _, k in pairs), np.uint8).copy()
    ops = np.zeros((n, FD_OPS_MAX), np.uint8)
    start = np.zeros(n, np.int32)
    # the merged recoder (throughput prep) and the two-pass one (latency front end)
    for fn in (harness.h_recode, harness.h_recode2):
        ops = np.zeros((n, FD_OPS_MAX), np.uint8)
        start = np.zeros(n, np.int32)
        fn(P(ops), P(start), P(S), P(K), ctypes.c_ulong(n))
        for i, (s, k) in enumerate(pairs):
            exp, st = expected_stream(oracle, s, k)
            assert start[i] == st, (fn, i, s, k)
            assert (ops[i] == exp).all(), (fn, i, s, k, np.nonzero(ops[i] != exp)[0][:8])
