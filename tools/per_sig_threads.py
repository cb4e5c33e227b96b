#!/usr/bin/env python3
"""fd_ed25519_verify (the per-signature drop-in, fd_ed25519.h:96-101) called
from T host threads at once: calls/s and per-call latency p50/p99 for
T = 1, 4, 16, 64.  Concurrent calls coalesce into shared batches on the
process-default engine (group commit, fd_ed25519_gpu_host.cpp), so
throughput grows with T while a lone caller's latency stays one round
trip.  One JSON line per T."""
import json
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import firedancer_amd as fa
    from firedancer_amd import corpus
    b = corpus.solana_txns(4096, seed=3)
    msgs = [b.msg(i) for i in range(len(b))]
    sigs = [b.sig(i) for i in range(len(b))]
    pubs = [b.pub(i) for i in range(len(b))]
    fa.verify(msgs[0], sigs[0], pubs[0])                 # engine up
    for T in (1, 4, 16, 64):
        per = max(200 // T, 20) if T > 1 else 400
        lat = [[] for _ in range(T)]
        bad = [0]

        def worker(t):
            for k in range(per):
                i = (t * per + k) % len(b)
                t0 = time.perf_counter()
                r = fa.verify(msgs[i], sigs[i], pubs[i])
                lat[t].append(time.perf_counter() - t0)
                if r != 0:
                    bad[0] += 1
        th = [threading.Thread(target=worker, args=(t,)) for t in range(T)]
        t0 = time.perf_counter()
        for x in th:
            x.start()
        for x in th:
            x.join()
        dt = time.perf_counter() - t0
        L = np.concatenate([np.array(x) for x in lat]) * 1e3
        print(json.dumps({"threads": T, "calls": T * per, "calls_per_s": T * per / dt,
                          "p50_ms": float(np.percentile(L, 50)), "p99_ms": float(np.percentile(L, 99)),
                          "rejected": bad[0], "msg": "C2 txn messages (1103/1167 B)"}), flush=True)


if __name__ == "__main__":
    main()
