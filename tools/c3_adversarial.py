#!/usr/bin/env python3
"""C3 (BASELINE.json configs[2] / north star): bit-exact accept/reject on
a 10M-signature adversarial corpus.

The corpus is built in chunks (seeded; 90% valid, 10% invalid split over
corpus.CASES: bit flips, S = L / L+1 / top byte >= 0x11, the early-accept
S pattern, non-canonical A/R, the 14 small-order encodings as A, R and
both, off-curve A/R, mixed-order A, x=0 with the sign bit) plus the three
SURVEY Q2 vectors.  Every chunk is verified by the engine on the GPU and
by the reference's own fd_ed25519_verify (oracle/_ref/libfdref.so, all
host threads); the codes must agree exactly, signature by signature.
Prints one progress line per chunk and a final JSON summary."""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from firedancer_amd import corpus  # noqa: E402

Q2 = corpus.Q2_VECTORS


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--total", type=int, default=10_000_000)
    ap.add_argument("--chunk", type=int, default=1_000_000)
    ap.add_argument("--msg-sz", type=int, default=128)
    ap.add_argument("--shape", choices=["packed", "txn"], default="packed",
                    help="packed: sig|pub|msg of --msg-sz; txn: 1232-byte Solana legacy txns (msg 1167/1103 B, C2 shape)")
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--schedules", default="pool,uniform,quad",
                    help="DSM schedules every chunk is verified under (all must match the reference)")
    a = ap.parse_args()
    import firedancer_amd as fa
    from firedancer_amd import corpus

    ref = ctypes.CDLL(os.path.join(ROOT, "oracle", "_ref", "libfdref.so"))
    P = lambda x: x.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    per_sig = corpus.TXN_MTU if a.shape == "txn" else 96 + a.msg_sz
    eng = fa.Engine(0, max_sigs=a.chunk + 8, max_blob=a.chunk * per_sig + 4096, depth=1)
    ncase = len(corpus.CASES)
    agree = np.zeros(ncase, np.int64)
    seen = np.zeros(ncase, np.int64)
    hist = {}
    mism = 0
    sched_mism = {}
    done = 0
    t_gen = t_gpu = t_ref = 0.0
    k = 0
    while done < a.total:
        n = min(a.chunk, a.total - done)
        t0 = time.time()
        if a.shape == "txn":
            b = corpus.adversarial_txns(n, seed=300 + k, invalid_frac=0.1, nthreads=a.threads)
        else:
            b = corpus.adversarial(n, a.msg_sz, seed=100 + k, invalid_frac=0.1, nthreads=a.threads)
        if k == 0:
            q = corpus.from_triples([(bytes.fromhex(m), bytes.fromhex(s), bytes.fromhex(p)) for m, s, p in Q2])
            b = corpus.concat([b, q])
        t1 = time.time()
        gots = {}
        for sch in a.schedules.split(","):
            eng.dsm_pool_min = 0 if sch == "pool" else 1 << 62
            eng.dsm_quad_max = 1 << 62 if sch == "quad" else 0
            eng.dsm_oct_max = 1 << 62 if sch == "oct" else 0
            gots[sch] = eng.verify_packed(b.blob, b.desc)
        got = gots[a.schedules.split(",")[0]]
        t2 = time.time()
        sig, pub, data, off, sz = b.flat()
        exp = np.zeros(len(b), np.int32)
        ref.ref_verify_batch(ctypes.c_uint64(len(b)), P(sig), P(pub), P(data), P(off), P(sz), P(exp), a.threads)
        t3 = time.time()
        t_gen += t1 - t0
        t_gpu += t2 - t1
        t_ref += t3 - t2
        lab = b.label.astype(np.int64)
        eq = got == exp
        mism += int((~eq).sum())
        for sch, g in gots.items():
            sched_mism[sch] = sched_mism.get(sch, 0) + int((g != exp).sum())
        np.add.at(seen, lab, 1)
        np.add.at(agree, lab, eq.astype(np.int64))
        uniq, cnts = np.unique(np.stack([lab, exp]), axis=1, return_counts=True)
        for c, cnt in zip(uniq.T, cnts):
            key = f"{corpus.CASES[int(c[0])]}:{int(c[1])}"
            hist[key] = hist.get(key, 0) + int(cnt)
        if k == 0:
            assert all(list(g[-3:]) == [fa.ERR_MSG] * 3 for g in gots.values()) and list(exp[-3:]) == [fa.ERR_MSG] * 3
        done += n
        k += 1
        print(f"chunk {k}: {done} sigs, mismatches so far {mism} {sched_mism}, gen {t1 - t0:.1f}s gpu {t2 - t1:.2f}s ref {t3 - t2:.1f}s",
              flush=True)
    res = {"config": "C3 adversarial corpus (BASELINE.json configs[2])", "signatures": int(seen.sum()),
           "mismatches": mism, "bit_exact": mism == 0 and not any(sched_mism.values()),
           "shape": a.shape, "msg_sz": [1103, 1167] if a.shape == "txn" else a.msg_sz,
           "mismatches_by_dsm_schedule": sched_mism,
           "per_case": {corpus.CASES[c]: {"n": int(seen[c]), "agree": int(agree[c])} for c in range(ncase)},
           "reference_codes_by_case": hist,
           "checker": "reference fd_ed25519_verify (AVX2 build, oracle/_ref/libfdref.so)",
           "seconds": {"generate": t_gen, "gpu_verify_pcie_incl": t_gpu, "reference_cpu": t_ref},
           "reference_cpu_threads": a.threads}
    print(json.dumps(res), flush=True)
    sys.exit(0 if res["bit_exact"] else 1)


if __name__ == "__main__":
    main()
