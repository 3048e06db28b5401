"""Per-upload timeline of the precompute from a rocpd database (tools/gpu.sh pre): for every upload (k_cellprep to the
last kernel before the next upload) its span, the kernels' busy time, and the largest gaps between consecutive
kernels with the kernels either side -- where the event-timed precompute_ms exceeds the sum of its kernels.
  python tools/ktimeline.py run_results.db [ngaps]"""
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
ngaps = int(sys.argv[2]) if len(sys.argv) > 2 else 8
cols = [r[1] for r in db.execute("pragma table_info(kernels)")]
name_col = "kernel_name" if "kernel_name" in cols else "name"
ks = [(s, e, n.split("(")[0].replace("void ", "")) for n, s, e in db.execute(f"select {name_col}, start, end from kernels")]
ks.sort()
starts = [i for i, k in enumerate(ks) if k[2] == "k_cellprep"]
for u, i0 in enumerate(starts):
    i1 = starts[u + 1] if u + 1 < len(starts) else len(ks)
    seg = ks[i0:i1]
    span = seg[-1][1] - seg[0][0]
    busy = sum(e - s for s, e, _ in seg)
    gaps = sorted(((seg[j + 1][0] - seg[j][1], seg[j][2], seg[j + 1][2]) for j in range(len(seg) - 1)), reverse=True)
    print(f"upload {u}: {len(seg)} kernels, span {span / 1e6:.2f} ms, busy {busy / 1e6:.2f} ms, "
          f"gaps {(span - busy) / 1e6:.2f} ms")
    for g, a, b in gaps[:ngaps]:
        print(f"   gap {g / 1e3:9.1f} us  {a} -> {b}")
