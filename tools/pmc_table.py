"""Per-kernel totals of every counter in rocprofv3 PMC output directories (rocpd .db or counter_collection.csv).

    python tools/pmc_table.py gpurun_out/pmc/*/ [--kernels k_ma,k_rpkt]
"""
import collections
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import load  # noqa: E402


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    want = None
    for a in sys.argv[1:]:
        if a.startswith("--kernels="):
            want = a.split("=", 1)[1].split(",")
    table = collections.defaultdict(dict)
    for d in args:
        import sqlite3

        names = set()
        for f in glob.glob(os.path.join(d, "**", "*.db"), recursive=True):
            names |= {r[0] for r in sqlite3.connect(f).execute("select distinct counter_name from counters_collection")}
        for c in sorted(names):
            agg, n = load(d, c)
            for k, v in agg.items():
                table[k][c] = (v, n[k])
    for k in sorted(table):
        if want and not any(k.startswith(w) for w in want):
            continue
        print(k)
        for c, (v, n) in sorted(table[k].items()):
            print(f"   {c:32s} total {v:14.6e}  launches {n:5d}  per launch {v / max(n, 1):14.6e}")


if __name__ == "__main__":
    main()
