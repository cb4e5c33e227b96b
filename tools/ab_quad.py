"""A/B of library variants on the latency schedule: quad-DSM HIP-event ms
of a lone 4096-signature C2 launch and one C2 ring point (depth 8, window
6, feeder, PCIe incl.) per variant, rounds interleaved.
usage: FD_ED25519_LIB is set per variant by this script:
python tools/ab_quad.py lib1.so lib2.so ... [--rounds R] [--nb NB]"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, os, sys
import numpy as np
sys.path.insert(0, %r)
import torch
import firedancer_amd as fa
from firedancer_amd import corpus
import bench
nb = int(sys.argv[1])
base = corpus.solana_txns(65536, seed=1000, nthreads=16)
dev = torch.device("cuda", 0)
s = torch.cuda.current_stream(dev).cuda_stream
n = 4096
d = base.desc[:n].copy()
hi = int(max((d["msg_off"] + d["msg_sz"]).max(), d["sig_off"].max() + 64))
blob = np.ascontiguousarray(base.blob[:hi])
d_blob = torch.from_numpy(np.concatenate([blob, np.zeros(64, np.uint8)])).to(dev)
d_desc = torch.from_numpy(d.view(np.uint8).copy()).to(dev)
d_out = torch.zeros(n, dtype=torch.int32, device=dev)
eng = fa.Engine(0, max_sigs=1 << 14, max_blob=1 << 26, depth=1)
for _ in range(5):
    eng.verify_dev_timed(n, d_blob.data_ptr(), len(blob), d_desc.data_ptr(), d_out.data_ptr(), s)
ks = np.array([eng.verify_dev_timed(n, d_blob.data_ptr(), len(blob), d_desc.data_ptr(), d_out.data_ptr(), s) for _ in range(40)])
acc = int((d_out == 0).sum().item())
eng.close()
r = bench.ring_stream(fa, base, 0, nb, 8, window=6)
print(json.dumps({"lib": os.environ.get("FD_ED25519_LIB", "default"), "accepted": acc,
                  "front_ms": round(float(np.median(ks[:, 0])), 4), "dsm_ms": round(float(np.median(ks[:, 3])), 4),
                  "ring_Mps": round(r["pcie_inclusive_verifies_per_s"] / 1e6, 2), "p50": round(r["p50_ms"], 3),
                  "p99": round(r["p99_ms"], 3), "ok": r["codes_ok"]}), flush=True)
""" % ROOT


def main():
    libs = [a for a in sys.argv[1:] if not a.startswith("--")]
    rounds, nb = 2, 2000
    if "--rounds" in sys.argv:
        rounds = int(sys.argv[sys.argv.index("--rounds") + 1])
    if "--nb" in sys.argv:
        nb = int(sys.argv[sys.argv.index("--nb") + 1])
    libs = [l for l in libs if not l.isdigit()]
    for _ in range(rounds):
        for lib in libs:
            env = dict(os.environ, FD_ED25519_LIB=os.path.abspath(lib))
            r = subprocess.run([sys.executable, "-u", "-c", CHILD, str(nb)], env=env, capture_output=True, text=True, timeout=300)
            if r.returncode:
                print("FAILED", lib, r.stderr[-2000:], flush=True)
                sys.exit(1)
            print(r.stdout.strip(), flush=True)


if __name__ == "__main__":
    main()
