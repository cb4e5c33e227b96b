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

Q2 = [("562c7b301299d47deefe44c5368b77333c214b79b3e7dc03b091f0add168c0910740ac7544423faa742c3ba3d5286c624e1c5174ae4ccad097bea9f3c3cc197f33b0c640b71ae479e30fb2b7159bfb099c9780aa80fff0c1ea9682838b906f8677ea561bef530df8f714bea2b6eeb81b7b468ab64220d9d62a00a557e66bb35d",
       "a53f00568d07e4944ee86da222b258beae6d8353024faf57de1fa83b05eea496267f66788337eab61e0d36da454c46700ad217fb3cb08d3d016548e4ff5be803",
       "5bba42a60de96030d8f6a85dc5809e3f39a210671f50ee0ffdab810e18725a49"),
      ("b594272285085ae80737ae28cf824783a8788d96d301ef3376d5f6de6599498fe92ab86784c593a3d42802cb97dcd15797351268f765787d68e4b6053cef065acc426921518d814afde0ca82fd788941a87e9468af2070c05755a2caeb6bdd34b8d108fe1ae96d59f8017eb0fe18c1a6da300403730cc3344d8cf5ecdba1bce9",
       "588e6a12357767161aae6b35a7768481883861dcb399c0929ba2319214871d93895b3ab2404066f4e92dba7c688dbca7874ef5c16bedcb1efc6eb50560fe3602",
       "a8c5f0b9a0cad87801e0e550c7b4cda39c96cc31b6de89123437e41c3f42ccfe"),
      ("fc2f6a47b996987a34e02bc58cc0e2f84144f1fa4a07d2964f2695e7daecdf8c1bb177623f9fe1d12b12a087383fa17153234d17507d1d45b5e009f968528efd7e51c1781977306ae975fee54e1665da6896fc2d53ce9ea9340282bbae55102db2dbaffb5798b0874037889b445e8b00afeeb1ad12f53e389f5cd7bc238bd4c9",
       "f064a139d45ec0994e332d79364ddd8c2894a3a9b97b571e864efe0cf2fbae0055b9ce729e97564fe0bf3444b29719f1908388a5ff1807355cff0a69561fb003",
       "1935951cae485585719b256b1132ccbc729da20b718cfe2950c18dcdd82bbd71")]


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
