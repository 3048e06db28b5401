"""Kernel statistics (the rocprofv3 --stats kernel_stats.csv columns) from a rocprofv3 rocpd database.

usage: python tools/rocpd_stats.py gpurun_out/prof/run_results.db > profiles/rNN_kernel_stats.csv
"""
import math
import sqlite3
import sys
from collections import defaultdict

db = sqlite3.connect(sys.argv[1])
cols = [r[1] for r in db.execute("pragma table_info(kernels)")]
name_col = "kernel_name" if "kernel_name" in cols else "name"
rows = db.execute(f"select {name_col}, start, end from kernels").fetchall()
d = defaultdict(list)
for name, s, e in rows:
    d[name].append(e - s)
total = sum(sum(v) for v in d.values())
print('"Name","Calls","TotalDurationNs","AverageNs","Percentage","MinNs","MaxNs","StdDev"')
for name, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    n = len(v)
    tot = sum(v)
    avg = tot / n
    sd = math.sqrt(sum((x - avg) ** 2 for x in v) / n)
    print(f'"{name}",{n},{tot},{avg:.6f},{100.0 * tot / total:.2f},{min(v)},{max(v)},{sd:.6f}')
