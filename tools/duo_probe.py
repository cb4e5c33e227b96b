"""Quad vs duo latency DSM: per-kernel HIP-event ms of one 4096-signature
C2 launch (HBM-resident) per schedule, then C2 ring points (feeder, PCIe
incl.) per (schedule, cu_groups, depth, window).
python tools/duo_probe.py [nb]"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import firedancer_amd as fa
    from firedancer_amd import corpus
    import bench
    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
    base = corpus.solana_txns(65536, seed=1000, nthreads=16)
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream(dev).cuda_stream
    for n in (4096, 8192):
        d = base.desc[:n].copy()
        hi = int(max((d["msg_off"] + d["msg_sz"]).max(), d["sig_off"].max() + 64))
        blob = np.ascontiguousarray(base.blob[:hi])
        d_blob = torch.from_numpy(np.concatenate([blob, np.zeros(64, np.uint8)])).to(dev)
        d_desc = torch.from_numpy(d.view(np.uint8).copy()).to(dev)
        d_out = torch.zeros(n, dtype=torch.int32, device=dev)
        for sched in (fa.LAT_QUAD, fa.LAT_DUO):
            eng = fa.Engine(0, max_sigs=1 << 14, max_blob=1 << 26, depth=1)
            eng.lat_dsm = sched
            for _ in range(5):
                eng.verify_dev_timed(n, d_blob.data_ptr(), len(blob), d_desc.data_ptr(), d_out.data_ptr(), s)
            ks = np.array([eng.verify_dev_timed(n, d_blob.data_ptr(), len(blob), d_desc.data_ptr(), d_out.data_ptr(), s)
                           for _ in range(30)])
            print(json.dumps({"n": n, "lat_dsm": sched, "accepted": int((d_out == 0).sum().item()),
                              "kernel_ms": {k: round(float(v), 4) for k, v in zip(fa.Engine.KERNELS, ks.mean(0))},
                              "kernel_ms_min": {k: round(float(v), 4) for k, v in zip(fa.Engine.KERNELS, ks.min(0))}}),
                  flush=True)
            eng.close()
    pts = [(fa.LAT_QUAD, 4, 8, 6), (fa.LAT_DUO, 8, 8, 6), (fa.LAT_DUO, 8, 8, 7), (fa.LAT_DUO, 8, 8, 8),
           (fa.LAT_DUO, 4, 8, 6), (fa.LAT_DUO, 4, 8, 8)]
    for sched, groups, depth, window in pts:
        r = bench.ring_stream(fa, base, 0, nb, depth, groups=groups, window=window, lat_dsm=sched)
        print(json.dumps({k: r[k] for k in ("lat_dsm", "cu_groups", "ring_depth", "window", "pcie_inclusive_verifies_per_s",
                                            "p50_ms", "p99_ms", "p999_ms", "submit_to_done_p99_ms", "codes_ok")}), flush=True)


if __name__ == "__main__":
    main()
