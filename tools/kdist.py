"""Per-kernel launch-duration distribution from a rocpd database: calls, total ms, and the 10/50/90/99th percentile
and max of the launch time in microseconds (which kernels have a per-launch floor, which a tail).

  python3 tools/kdist.py DB [N]
"""
import sqlite3
import sys
from collections import defaultdict

import numpy as np

db = sqlite3.connect(sys.argv[1])
cols = [r[1] for r in db.execute("pragma table_info(kernels)")]
name_col = "kernel_name" if "kernel_name" in cols else "name"
d = defaultdict(list)
for name, s, e in db.execute(f"select {name_col}, start, end from kernels"):
    d[name.split("(")[0].replace("void ", "")].append(e - s)
n = int(sys.argv[2]) if len(sys.argv) > 2 else 16
print(f"{'kernel':44s} {'calls':>6s} {'total ms':>10s} {'p10 us':>8s} {'p50 us':>8s} {'p90 us':>8s} {'p99 us':>8s} {'max us':>9s}")
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1]))[:n]:
    a = np.array(v, dtype=np.float64) / 1e3
    p = np.percentile(a, [10, 50, 90, 99])
    print(f"{k[:44]:44s} {len(a):6d} {a.sum() / 1e3:10.2f} {p[0]:8.1f} {p[1]:8.1f} {p[2]:8.1f} {p[3]:8.1f} {a.max():9.1f}")
