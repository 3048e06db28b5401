"""Summarise rocprofv3 PMC counter CSVs into the per-launch HBM traffic bench.py reports as roofline.traffic.

    python tools/pmc_summary.py --fetch DIR1 --write DIR2 --packets P --ngrid G --nts T --out profiles/pmc_r01.json

DIR1 / DIR2 are rocprofv3 `--pmc FETCH_SIZE` / `--pmc WRITE_SIZE` output directories (separate passes: the two
counters do not fit one TCC pass on gfx950) of the same bench command.  FETCH_SIZE and WRITE_SIZE are in KiB;
on gfx950 FETCH_SIZE reports half the bytes of wide streaming reads, so it is doubled
(/opt/skills/guides/MI355X_MICROARCH.md, HBM section).  Output: per kernel, launches, and HBM bytes per launch.
"""
import argparse
import collections
import csv
import glob
import json
import os
import sqlite3


def load(d, counter):
    agg = collections.defaultdict(float)
    launches = collections.Counter()
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        rows += [(r["Kernel_Name"], r["Counter_Name"], r["Counter_Value"]) for r in csv.DictReader(open(f))]
    for f in glob.glob(os.path.join(d, "**", "*.db"), recursive=True):  # rocprofv3 >= 7.2 default (rocpd sqlite)
        rows += sqlite3.connect(f).execute(
            "select kernel_name, counter_name, value from counters_collection").fetchall()
    for kname, cname, value in rows:
        if cname != counter:
            continue
        name = kname.split("(")[0].replace("void ", "")
        agg[name] += float(value)
        launches[name] += 1
    return agg, launches


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--packets", type=int, required=True)
    ap.add_argument("--ngrid", type=int, required=True)
    ap.add_argument("--nts", type=int, required=True)
    ap.add_argument("--steps", type=int, default=1, help="transport steps in the profiled run (warmup included)")
    ap.add_argument("--vpkt", type=int, default=0, help="observer directions of the profiled run (bench.py --vpkt)")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    fetch, nf = load(a.fetch, "FETCH_SIZE")
    write, nw = load(a.write, "WRITE_SIZE")
    kernels = {}
    for name in sorted(set(fetch) | set(write)):
        n = max(nf[name], nw[name], 1)
        fb = 2.0 * fetch.get(name, 0.0) * 1024.0  # gfx950: FETCH_SIZE counts half of wide reads
        wb = write.get(name, 0.0) * 1024.0
        kernels[name] = {"launches": n, "fetch_bytes_per_launch": fb / n, "write_bytes_per_launch": wb / n,
                         "hbm_bytes_per_launch": (fb + wb) / n,
                         "hbm_bytes_per_step": (fb + wb) / a.steps}
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from artis_amd import engine_src_sha

    out = {"engine_src_sha": engine_src_sha(), "packets": a.packets, "ngrid": a.ngrid, "nts": a.nts,
           "vpkt": a.vpkt, "steps": a.steps,
           "correction": "FETCH_SIZE x2 (gfx950), KiB -> bytes", "kernels": kernels}
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    for name, k in sorted(kernels.items(), key=lambda kv: -kv[1]["hbm_bytes_per_step"])[:8]:
        print(f"{name:40s} launches {k['launches']:6d}  HBM/launch {k['hbm_bytes_per_launch']:.3e} B")


if __name__ == "__main__":
    main()
