#!/usr/bin/env python3
"""The shader clock the latency DSMs run at (fd_ed25519_gpu_dsm_clock):
single-signature calls (the eight-lane DSM) one after another, and lone
4,096-signature batches (the quad DSM), each on an otherwise idle device.
Separates the per-signature latency's clock from its instruction count.
Variant libraries (FD_ED25519_LIB) A/B the oct DSM's main loop by its
cycles per wave (one wave per single-signature call).
usage: oct_clock.py [calls]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    import firedancer_amd as fa
    from firedancer_amd import corpus
    b = corpus.solana_txns(4096, seed=1000, nthreads=16)
    e = fa.Engine(0, 4096, 1 << 24, depth=1)
    out = {}
    for name, n, reps in (("oct_n1", 1, calls), ("quad_n4096", 4096, max(calls // 10, 20))):
        d = b.desc[:n].copy()
        hi = int(max((d["msg_off"] + d["msg_sz"]).max(), d["sig_off"].max() + 64, d["pub_off"].max() + 32))
        blob = np.ascontiguousarray(b.blob[:hi])
        e.verify_packed(blob, d)
        e.dsm_clock(clear=True)
        t = []
        for _ in range(reps):
            t0 = time.perf_counter()
            got = e.verify_packed(blob, d)
            t.append(time.perf_counter() - t0)
        c = e.dsm_clock()
        k = "oct" if n <= e.dsm_oct_max else "quad"
        out[name] = {"kernel": k, "waves": c[k]["waves"], "ghz": c[k]["ghz"], "loop_cycles_per_wave": c[k]["cycles_per_wave"],
                     "loop_us_per_wave": c[k]["us_per_wave"], "call_p50_ms": float(np.median(t) * 1e3),
                     "accepted": int((got == 0).sum())}
    print(json.dumps(out), flush=True)
    e.close()


if __name__ == "__main__":
    main()
