#!/usr/bin/env python3
"""Kernel stats (the rocprofv3 --stats kernel_stats.csv columns) from a
rocprofv3 SQLite results database (rocpd, the default output format):
python3 tools/rocpd_stats.py <results.db> > <kernel_stats.csv>"""
import sqlite3
import statistics
import sys
from collections import defaultdict


def main():
    c = sqlite3.connect(sys.argv[1])
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    d = defaultdict(list)
    for k, s, e in c.execute(f"select {name}, start, end from kernels"):
        d[k].append(e - s)
    tot = sum(sum(v) for v in d.values())
    print('"Name","Calls","TotalDurationNs","AverageNs","Percentage","MinNs","MaxNs","StdDev"')
    for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
        sd = statistics.pstdev(v) if len(v) > 1 else 0.0
        print(f'"{k}",{len(v)},{sum(v)},{sum(v) / len(v):.6f},{100.0 * sum(v) / tot:.2f},{min(v)},{max(v)},{sd:.6f}')


if __name__ == "__main__":
    main()
