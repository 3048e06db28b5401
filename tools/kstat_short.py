"""Short kernel table from a rocpd database: name (without arguments), calls, total ms, average ms."""
import sqlite3
import sys
from collections import defaultdict

db = sqlite3.connect(sys.argv[1])
cols = [r[1] for r in db.execute("pragma table_info(kernels)")]
name_col = "kernel_name" if "kernel_name" in cols else "name"
d = defaultdict(list)
for name, s, e in db.execute(f"select {name_col}, start, end from kernels"):
    d[name.split("(")[0].replace("void ", "")].append(e - s)
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1]))[:n]:
    print(f"{k[:44]:44s} {len(v):6d} {sum(v) / 1e6:10.2f} ms {sum(v) / len(v) / 1e6:9.3f} ms")
