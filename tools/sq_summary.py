"""Summarise a rocprofv3 SQ-counter pass (tools/gpu_sq.sh) per kernel:

    python tools/sq_summary.py gpurun_out/sq/db > profiles/<tag>_sq_counters.txt

SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES is the fraction of a wave's cycles it issues VALU instructions (times the
waves per SIMD: the SIMD's VALU occupancy); instruction counts are wave instructions summed over the launches.
"""
import collections
import glob
import os
import sqlite3
import sys


def main(d):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(os.path.join(d, "**", "*.db"), recursive=True):
        for kname, cname, value in sqlite3.connect(f).execute(
                "select kernel_name, counter_name, value from counters_collection"):
            agg[kname.split("(")[0].replace("void ", "")][cname] += float(value)
    for k, c in sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0))[:8]:
        wc = max(c.get("SQ_WAVE_CYCLES", 0), 1)
        print(f"{k:14s} VALU-active/wave-cycles {c.get('SQ_ACTIVE_INST_VALU', 0) / wc:.3f}  any-active/wave-cycles "
              f"{c.get('SQ_ACTIVE_INST_ANY', 0) / wc:.3f}  insts VALU {c.get('SQ_INSTS_VALU', 0):.3e} SALU "
              f"{c.get('SQ_INSTS_SALU', 0):.3e} LDS {c.get('SQ_INSTS_LDS', 0):.3e} VMEM {c.get('SQ_INSTS_VMEM', 0):.3e}")


if __name__ == "__main__":
    main(sys.argv[1])
