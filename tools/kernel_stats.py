"""rocprofv3 (rocpd sqlite, ROCm >= 7.2 default output) -> kernel statistics CSV like --stats' kernel_stats.csv:
Name, Calls, TotalDurationNs, AverageNs, Percentage, plus VGPRs / scratch bytes / LDS bytes per kernel.

usage: python tools/kernel_stats.py <dir with *.db> <out.csv>
"""
import csv
import glob
import os
import sqlite3
import sys


def main(d, out):
    rows = {}
    for f in glob.glob(os.path.join(d, "**", "*.db"), recursive=True):
        db = sqlite3.connect(f)
        for name, dur, scratch, lds in db.execute("select name, duration, scratch_size, lds_size from kernels"):
            r = rows.setdefault(name, [0, 0, 0, 0])
            r[0] += 1
            r[1] += dur
            r[2] = max(r[2], scratch or 0)
            r[3] = max(r[3], lds or 0)
        vg = dict(db.execute("select distinct k.name, s.arch_vgpr_count from kernels k join kernel_symbols s "
                             "on k.kernel_id = s.kernel_id"))
    total = sum(r[1] for r in rows.values()) or 1
    with open(out, "w", newline="") as fo:
        w = csv.writer(fo)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "ArchVGPR", "ScratchBytes", "LDSBytes"])
        for name, r in sorted(rows.items(), key=lambda kv: -kv[1][1]):
            w.writerow([name, r[0], r[1], r[1] / r[0], 100.0 * r[1] / total, vg.get(name, ""), r[2], r[3]])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
