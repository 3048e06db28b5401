"""Compare the first-pass NLTE rate matrices dumped by the engine (ARTIS_GPU_NL_DUMP=prefix) and by the oracle
(ORACLE_NL_DUMP=prefix): per element, the largest relative differences of the matrix columns, b, the LTE
normalisation and the solved populations.  Diagnostics only."""
import os
import sys

import numpy as np


def main(prefix, npass=1):
    for p in range(npass):
        if os.path.exists(f"{prefix}_p{p}_gpu.bin"):
            print(f"--- pass {p}")
            compare(f"{prefix}_p{p}")


def compare(prefix):
    with open(prefix + "_gpu.bin", "rb") as f:
        ne, cell1, cell2, nl, ntg = np.frombuffer(f.read(20), np.int32)
        el_D = np.frombuffer(f.read(4 * ne), np.int32)
        status = np.frombuffer(f.read(4 * ne), np.int32)
        A = np.frombuffer(f.read(8 * cell2), np.float64)
        b = np.frombuffer(f.read(8 * cell1), np.float64)
        nrm = np.frombuffer(f.read(8 * cell1), np.float64)
        pv = np.frombuffer(f.read(8 * cell1), np.float64)
    o1 = o2 = 0
    for e in range(ne):
        D = int(el_D[e])
        if D == 0:
            continue
        fn = f"{prefix}_ora_e{e}.bin"
        Ag = A[o2:o2 + D * D].reshape(D, D).T  # [row, col]
        bg, ng, pg = b[o1:o1 + D], nrm[o1:o1 + D], pv[o1:o1 + D]
        o1 += D
        o2 += D * D
        if not os.path.exists(fn):
            print(f"element {e}: D {D} no oracle dump (abundance 0?) gpu status {status[e]}")
            continue
        with open(fn, "rb") as f:
            Do, so = np.frombuffer(f.read(8), np.int32)
            Ao = np.frombuffer(f.read(8 * D * D), np.float64).reshape(D, D).T
            bo = np.frombuffer(f.read(8 * D), np.float64)
            no = np.frombuffer(f.read(8 * D), np.float64)
            po = np.frombuffer(f.read(8 * D), np.float64)
        assert Do == D, (Do, D)
        scale = np.maximum(np.abs(Ao).max(axis=0), 1e-300)
        colerr = (np.abs(Ag - Ao) / scale).max(axis=0)
        rel = lambda g, o: float(np.max(np.abs(g - o) / np.maximum(np.abs(o), 1e-300)))  # noqa: E731
        worst = np.argsort(colerr)[::-1][:4]
        print(f"element {e}: D {D} status gpu {status[e]} oracle {so}; A col err max {colerr.max():.2e} at cols "
              f"{worst.tolist()} ({colerr[worst]}); b {rel(bg, bo):.2e} norm {rel(ng, no):.2e} pv {rel(pg, po):.2e}")
        if colerr.max() > 1e-8:
            c = int(worst[0])
            r = int(np.argmax(np.abs(Ag[:, c] - Ao[:, c])))
            print(f"   col {c} row {r}: gpu {Ag[r, c]:.6e} oracle {Ao[r, c]:.6e}; diag gpu {Ag[c, c]:.6e} oracle "
                  f"{Ao[c, c]:.6e}; norm gpu {ng[c]:.6e} oracle {no[c]:.6e}")
        if rel(pg, po) > 1e-6:
            k = int(np.argmax(np.abs(pg - po) / np.maximum(np.abs(po), 1e-300)))
            print(f"   pv[{k}]: gpu {pg[k]:.6e} oracle {po[k]:.6e}; sum gpu {pg.sum():.6e} oracle {po.sum():.6e} b0 {bo[0]:.6e}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 4)
