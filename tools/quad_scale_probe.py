import sys, os, numpy as np
sys.path.insert(0, os.getcwd())
import firedancer_amd as fa
from firedancer_amd import corpus
base = corpus.solana_txns(1 << 20, seed=1000, nthreads=16)
e = fa.Engine(0, 1 << 20, len(base.blob) + 4096, depth=1)
for pm, qm in ((1 << 62, 1 << 62),):
    e.dsm_pool_min, e.dsm_quad_max = pm, qm
    for n in (4096, 16384, 65536, 262144, 1 << 20):
        got = e.verify_packed(base.blob, base.desc[:n])
        print(n, "rejected", int((got != 0).sum()), flush=True)
e.close()
