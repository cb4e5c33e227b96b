#!/usr/bin/env python3
"""Per-kernel register / LDS / occupancy table of the product kernels
(compiler resource-usage remarks for gfx950), with the resource that caps
each kernel's waves per SIMD.  CPU only (cross-compiles the kernels file).

usage: python3 tools/kernel_resources.py [rocprof kernel_trace.csv]
  (the optional trace adds what the runtime reported at dispatch)"""
import collections
import csv
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "firedancer_amd", "csrc", "fd_ed25519_gpu_kernels.hip")
LDS_CU = 160 * 1024
VGPR_SIMD = 512
WAVE_SLOTS = 8


def remarks():
    with tempfile.TemporaryDirectory() as d:
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
               "-I" + os.path.join(ROOT, "firedancer_amd", "csrc"), "-I" + os.path.join(ROOT, "include"),
               "--cuda-device-only", "-c", SRC, "-o", os.path.join(d, "k.o"), "-Rpass-analysis=kernel-resource-usage"]
        out = subprocess.run(cmd, capture_output=True, text=True).stderr
    ks, cur = collections.OrderedDict(), None
    for line in out.splitlines():
        m = re.search(r"remark: (.*?) \[-Rpass", line)
        if not m:
            continue
        t = m.group(1).strip()
        if t.startswith("Function Name:"):
            cur = t.split(":", 1)[1].strip()
            ks[cur] = {}
        elif cur and ":" in t:
            k, v = t.split(":", 1)
            ks[cur][k.strip()] = v.strip()
    return ks


def main():
    ks = remarks()
    trace = {}
    if len(sys.argv) > 1:
        for r in csv.DictReader(open(sys.argv[1])):
            n = r["Kernel_Name"].split("(")[0]
            if n.startswith("fd_k") and n not in trace:
                trace[n] = r
    print("%-18s %5s %5s %6s %6s %8s %5s  %-10s %s" % ("kernel", "VGPR", "SGPR", "vspill", "sspill", "LDS/WG", "occ", "limit", "dispatch (rocprof)"))
    for n, v in ks.items():
        if not n.startswith("fd_k"):
            continue
        vg = int(v.get("VGPRs", 0)) + int(v.get("AGPRs", 0))
        lds = int(v.get("LDS Size [bytes/block]", 0))
        occ = int(v.get("Occupancy [waves/SIMD]", 0))
        alloc = (vg + 7) // 8 * 8
        by_v = VGPR_SIMD // max(alloc, 1)
        wgw = 1 if n in ("fd_k_dsm_quad", "fd_k_front") else 4   # waves per workgroup
        by_l = (LDS_CU // lds) * wgw // 4 if lds else WAVE_SLOTS
        limit = "+".join(x for x, y in (("VGPR", by_v), ("LDS", by_l)) if y == occ) or "waves"
        t = trace.get(n)
        extra = (f"wg {t['Workgroup_Size_X']}, grid {t['Grid_Size_X']}, scratch {t['Scratch_Size']}" if t else "")
        print("%-18s %5d %5s %6s %6s %8d %5d  %-10s %s" % (n, vg, v.get("SGPRs", "-"), v.get("VGPRs Spill", "?"),
                                                        v.get("SGPRs Spill", "?"), lds, occ, limit, extra))


if __name__ == "__main__":
    main()
