#!/usr/bin/env python3
"""Regenerate tests/golden/config_digests.json: the reference's own
per-signature codes (oracle/_ref/libfdref.so, the AVX2 fd_ed25519_verify
built in place from /root/reference by oracle/Makefile) over the
deterministic, seeded BASELINE-size corpora of SURVEY.md section 8d,
recorded as a SHA-256 digest of the int8 code vector plus a histogram.

The corpora are regenerated on the GPU box from their seeds
(firedancer_amd.corpus: numpy's seeded generator + the product's
deterministic host signer), so tests/test_gpu_configs.py can pin the
engine's codes to the reference even where the reference build is not
shipped; where it is, the tests also compare code by code.

  c1     1,048,576 x (128-byte msg), all valid                    (C1)
  c3c2   1,048,576 signatures of Solana-MTU txns (msg 1167/1103 B), 10 %
         corrupted over all 18 invalid cases                      (C3 at C2 shape)
  c4     one 256-byte / 442-byte message, n = 1..16 and 4096 signers,
         25 % of the signatures corrupted (signature/key cases only)  (C4)
  c3_10m the north star's 10M-signature adversarial corpus at C2 shape:
         10 chunks of 1,000,000 txn signatures (seeds 4200+k), 10 %
         corrupted over all 18 invalid cases, plus the three SURVEY Q2
         vectors after chunk 0 -- 10,000,003 signatures; a digest per
         chunk and the histogram of the whole                     (C3)

Runs only in the build container (needs the reference build)."""
import ctypes
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from firedancer_amd import corpus  # noqa: E402

C1 = {"n": 1 << 20, "msg_sz": 128, "seed": 4101}
C3C2 = {"n": 1 << 20, "seed": 4102, "invalid_frac": 0.1}
C4_SIZES = (256, 442)
C4_NS = list(range(1, 17)) + [4096]
C4_CASES = ["flip_R", "flip_S", "flip_pub", "S_eq_L", "S_eq_L1", "S_top_big", "S_q1_early_accept",
            "noncanon_A", "noncanon_R", "small_A", "small_R", "small_both", "offcurve_A", "offcurve_R",
            "mixed_order_A", "negzero_A", "negzero_R"]


def digest(codes):
    return hashlib.sha256(np.ascontiguousarray(codes, np.int8).tobytes()).hexdigest()


def hist(codes):
    u, c = np.unique(codes, return_counts=True)
    return {str(int(a)): int(b) for a, b in zip(u, c)}


def c1_batch(nthreads=8):
    return corpus.simple(C1["n"], C1["msg_sz"], seed=C1["seed"], nthreads=nthreads)


def c3c2_batch(nthreads=8):
    return corpus.adversarial_txns(C3C2["n"], seed=C3C2["seed"], invalid_frac=C3C2["invalid_frac"], nthreads=nthreads)


C3_10M = {"chunks": 10, "chunk": 1_000_000, "seed0": 4200, "invalid_frac": 0.1}
# the three SURVEY.md section 8c Q2 vectors (msg, sig, pub hex): valid
# signatures the reference rejects through its limb compare
Q2_VECTORS = corpus.Q2_VECTORS


def c3_10m_chunk(k, nthreads=8):
    """chunk k of the 10M C3 corpus (chunk 0 carries the three Q2 vectors at its end)"""
    b = corpus.adversarial_txns(C3_10M["chunk"], seed=C3_10M["seed0"] + k, invalid_frac=C3_10M["invalid_frac"],
                                nthreads=nthreads)
    if k == 0:
        q = corpus.from_triples([(bytes.fromhex(m), bytes.fromhex(s), bytes.fromhex(p)) for m, s, p in Q2_VECTORS])
        b = corpus.concat([b, q])
    return b


def c4_batch(msg_sz, n, nthreads=8):
    """(batch, shared msg, sig[n,64], pub[n,32]) for one C4 case"""
    b, msg, _, _ = corpus.single_msg(n, msg_sz, seed=5000 + 100 * n + msg_sz, nthreads=nthreads)
    corpus.corrupt(b, seed=6000 + 100 * n + msg_sz, invalid_frac=0.25, cases=C4_CASES)
    sig, pub, _, _, _ = b.flat()
    return b, bytes(msg), sig, pub


def ref_codes(L, b, threads=8):
    sig, pub, data, off, sz = b.flat()
    out = np.zeros(len(b), np.int32)
    P = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    L.ref_verify_batch(ctypes.c_ulong(len(b)), P(sig), P(pub), P(data), P(off), P(sz), P(out), threads)
    return out


def c3_10m(L, nthreads=8):
    chunks, tot, labels = [], {}, {}
    for k in range(C3_10M["chunks"]):
        b = c3_10m_chunk(k, nthreads)
        e = ref_codes(L, b, nthreads)
        chunks.append(digest(e))
        for a, c in hist(e).items():
            tot[a] = tot.get(a, 0) + c
        for a, c in hist(b.label).items():
            labels[a] = labels.get(a, 0) + c
        print(f"c3_10m chunk {k}: {len(b)} sigs {hist(e)}", flush=True)
    return dict(C3_10M, signatures=sum(tot.values()), chunk_digests=chunks, hist=tot, label_hist=labels)


def main():
    # (the product library is only the signer here; importing this module
    # from the GPU tests must not change how the library loads)
    L = ctypes.CDLL(os.path.join(ROOT, "oracle", "_ref", "libfdref.so"))
    if sys.argv[1:] == ["--only", "c3_10m"]:
        path = os.path.join(HERE, "config_digests.json")
        res = json.load(open(path))
        res["c3_10m"] = c3_10m(L, os.cpu_count() or 8)
        json.dump(res, open(path, "w"), indent=1)
        print(json.dumps(res["c3_10m"]["hist"]))
        return
    res = {"generator": "tests/golden/make_config_digests.py", "checker": "oracle/_ref/libfdref.so (reference AVX2 build)"}
    b = c1_batch()
    e = ref_codes(L, b)
    res["c1"] = dict(C1, digest=digest(e), hist=hist(e))
    del b
    b = c3c2_batch()
    e = ref_codes(L, b)
    res["c3c2"] = dict(C3C2, digest=digest(e), hist=hist(e), label_hist=hist(b.label))
    del b
    c4 = {}
    for sz in C4_SIZES:
        for n in C4_NS:
            b, _, _, _ = c4_batch(sz, n)
            e = ref_codes(L, b)
            c4[f"{sz}/{n}"] = {"codes": e.tolist()} if n <= 16 else {"digest": digest(e), "hist": hist(e)}
    res["c4"] = {"sizes": list(C4_SIZES), "ns": C4_NS, "cases": C4_CASES, "expected": c4}
    res["c3_10m"] = c3_10m(L)
    json.dump(res, open(os.path.join(HERE, "config_digests.json"), "w"), indent=1)
    print(json.dumps({k: v.get("hist") for k, v in res.items() if isinstance(v, dict) and "hist" in v}))


if __name__ == "__main__":
    main()
