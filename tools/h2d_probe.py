#!/usr/bin/env python3
"""H2D bandwidth from pinned host memory on one MI355X: one copy stream
against the same bytes split over 2 and 4 streams (do concurrent copies
engage more SDMA engines and get closer to the PCIe limit?).  One JSON
line.  usage: h2d_probe.py [MiB per copy (default 256)]"""
import json
import sys
import time

import torch


def run(nbytes, nstreams, reps=8):
    src = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    dst = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    sts = [torch.cuda.Stream() for _ in range(nstreams)]
    part = nbytes // nstreams
    for _ in range(2):
        for k, s in enumerate(sts):
            with torch.cuda.stream(s):
                dst[k * part:(k + 1) * part].copy_(src[k * part:(k + 1) * part], non_blocking=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        for k, s in enumerate(sts):
            with torch.cuda.stream(s):
                dst[k * part:(k + 1) * part].copy_(src[k * part:(k + 1) * part], non_blocking=True)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return reps * part * nstreams / dt / 1e9


def main():
    mib = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    n = mib << 20
    out = {"mib": mib}
    for ns in (1, 2, 4, 1, 2, 4):
        out.setdefault(f"streams_{ns}_GBps", []).append(round(run(n, ns), 2))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
