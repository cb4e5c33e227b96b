#!/usr/bin/env python3
"""Per-kernel issue split from one SQ counter pass (tools/gpu.sh pmcsq=<lib>):
VALU instructions per wave, cycles per VALU instruction per wave
(SQ_WAVE_CYCLES counts quad-cycles on gfx950, hence x4), the fraction of a
wave's cycles it issued VALU work and waited on an instruction dependency,
and the chip-wide VALU issue rate per SIMD-cycle (GRBM_GUI_ACTIVE summed over
8 XCDs).  usage: pmc_split.py <pmc dir> [...]"""
import collections
import csv
import sys


def main():
    for d in sys.argv[1:]:
        agg = collections.defaultdict(lambda: collections.defaultdict(list))
        for r in csv.DictReader(open(d + "/run_counter_collection.csv")):
            agg[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, c in sorted(agg.items()):
            if not k.startswith("fd_k"):
                continue
            m = {x: sum(v) / len(v) for x, v in c.items()}
            w = m["SQ_WAVES"]
            vi = m["SQ_INSTS_VALU"]
            wc = m["SQ_WAVE_CYCLES"] * 4
            clk = m["GRBM_GUI_ACTIVE"] / 8
            print(f'{d.rstrip("/").split("/")[-1]:22s} {k[:16]:16s} waves {w:8.0f} valu/wave {vi / w:9.0f} '
                  f'cyc/instr/wave {wc / vi:6.2f} valu_active {m["SQ_ACTIVE_INST_VALU"] / m["SQ_WAVE_CYCLES"]:.3f} '
                  f'wait_inst {m["SQ_WAIT_INST_ANY"] / m["SQ_WAVE_CYCLES"]:.3f} gui_cyc {clk:10.0f} '
                  f'issue/SIMD-cyc {vi / 1024 / clk:.3f}')


if __name__ == "__main__":
    main()
