"""Each launch of the named kernels in a rocpd database, in time order: start offset (ms from the first kernel) and
duration -- to tell the uploads of a multi-step run apart (e.g. level mode's warm-step and timed-step record builds).
  python tools/klaunches.py run_results.db k_ma_build k_marates k_cooling"""
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
cols = [r[1] for r in db.execute("pragma table_info(kernels)")]
name_col = "kernel_name" if "kernel_name" in cols else "name"
ks = sorted((s, e, n.split("(")[0].replace("void ", "")) for n, s, e in db.execute(f"select {name_col}, start, end from kernels"))
t0 = ks[0][0] if ks else 0
for s, e, n in ks:
    if any(n.startswith(p) for p in sys.argv[2:]):
        print(f"{(s - t0) / 1e6:12.1f} ms  {(e - s) / 1e6:10.2f} ms  {n}")
