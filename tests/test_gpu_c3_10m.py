"""The north star's bit-exactness bar on the GPU itself (BASELINE.json
north_star, configs[2]): 100 % agreement with the reference's
fd_ed25519_verify (src/ballet/ed25519/fd_ed25519_user.c:346-433, AVX2
build) on a 10M-signature adversarial corpus.

10,000,003 signatures at C2 shape (1232-byte Solana txns, messages of
1167 / 1103 bytes), 10 % corrupted over all 18 invalid cases of
firedancer_amd.corpus.CASES (bit flips, S = L / L+1 / top byte >= 0x11,
the early-accept S pattern, non-canonical A and R, the 14 small-order
encodings as A, R and both, off-curve A and R, a mixed-order key, x = 0
with the sign bit), plus the three SURVEY Q2 vectors, generated in ten
seeded chunks of 1,000,000 (tests/golden/make_config_digests.py).

Every chunk is verified under the DSM schedule the bench's throughput
launches use (pool), the one the C2 ring's 4096-signature batches use
(quad) and the per-signature drop-in's eight-lane one (oct, forced to the
chunk size), and every code of each is compared with the reference build
(oracle/_ref/libfdref.so, compiled in place from /root/reference and
shipped with the tree) and with the committed per-chunk digest of the
reference's codes (recorded in the build container)."""
import hashlib
import json
import os
import sys
import time

import numpy as np
import pytest

import firedancer_amd as fa
from conftest import GOLDEN, oracle_batch
from firedancer_amd import corpus

sys.path.insert(0, GOLDEN)
import make_config_digests as mcd  # noqa: E402

pytestmark = pytest.mark.gpu

NTH = min(16, os.cpu_count() or 8)
DIG = json.load(open(os.path.join(GOLDEN, "config_digests.json")))


def _digest(codes):
    return hashlib.sha256(np.ascontiguousarray(codes, np.int8).tobytes()).hexdigest()


def test_c3_10m_adversarial_every_code_equals_reference(ref):
    spec = DIG["c3_10m"]
    e = fa.Engine(0, 1 << 20, 1 << 30, depth=1)
    schedules = {"pool": (0, 0, 0), "quad": (1 << 62, 1 << 62, 0), "oct": (1 << 62, 0, 1 << 62)}   # (dsm_pool_min, dsm_quad_max, dsm_oct_max)
    total, mism, n_sigs = {}, {s: 0 for s in schedules}, 0
    cases_seen = set()
    t0 = time.time()
    try:
        for k in range(spec["chunks"]):
            b = mcd.c3_10m_chunk(k, NTH)
            cases_seen |= set(np.unique(b.label).tolist())
            exp = oracle_batch(ref, b, NTH)
            # the reference build on this box gives the codes recorded in the container
            assert _digest(exp) == spec["chunk_digests"][k], k
            for sched, (pool_min, quad_max, oct_max) in schedules.items():
                e.dsm_pool_min, e.dsm_quad_max, e.dsm_oct_max = pool_min, quad_max, oct_max
                got = e.verify_packed(b.blob, b.desc)
                bad = np.nonzero(got != exp)[0]
                mism[sched] += len(bad)
                assert len(bad) == 0, (k, sched, [(int(i), corpus.CASES[b.label[i]], int(exp[i]), int(got[i])) for i in bad[:8]])
                assert _digest(got) == spec["chunk_digests"][k], (k, sched)
            for a, c in zip(*np.unique(exp, return_counts=True)):
                total[str(int(a))] = total.get(str(int(a)), 0) + int(c)
            n_sigs += len(b)
            if k == 0:
                assert list(exp[-3:]) == [fa.ERR_MSG] * 3     # the Q2 vectors: rejected by the reference and the engine
            print(f"c3_10m chunk {k}: {n_sigs} signatures, mismatches {mism}, {time.time() - t0:.0f} s", flush=True)
    finally:
        e.close()
    assert n_sigs == spec["signatures"] == 10_000_003
    assert total == spec["hist"]
    assert cases_seen == set(range(len(corpus.CASES)))
    assert mism == {"pool": 0, "quad": 0, "oct": 0}
