#!/usr/bin/env python3
"""Codes of an adversarial corpus through a registered blob (the ring's
direct path) in 4,000-signature batches; prints a digest and the reject
histogram, for comparing engine knobs (run it once per setting)."""
import hashlib
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import firedancer_amd as fa
    from firedancer_amd import corpus
    adv = corpus.adversarial_txns(20000, seed=5)
    eng = fa.Engine(0, max_sigs=4096, max_blob=len(adv.blob) + 4096, depth=8)
    try:
        eng.register(adv.blob)
        out = np.concatenate([eng.verify_packed(adv.blob, adv.desc[s:s + 4000]) for s in range(0, len(adv), 4000)])
    finally:
        eng.close()
    print(json.dumps({"n": int(len(out)), "sha256": hashlib.sha256(out.astype(np.int32).tobytes()).hexdigest(),
                      "hist": {int(k): int(v) for k, v in zip(*np.unique(out, return_counts=True))}}))


if __name__ == "__main__":
    main()
