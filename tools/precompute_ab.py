"""Times the per-timestep precompute (artis_gpu_upload_cellstate) of the bench model alone: N uploads, the last
N-1 reported.  For A/B builds (ARTIS_GPU_SO=build/ab/<name>/libartis_gpu.so) and rocprofv3 kernel tables.
  python tools/precompute_ab.py [--uploads 4] [--ngrid 50] [--nts 10]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--uploads", type=int, default=4)
    ap.add_argument("--ngrid", type=int, default=50)
    ap.add_argument("--nts", type=int, default=10)
    args = ap.parse_args()
    import torch

    if not torch.cuda.is_available():
        raise SystemExit("needs a GPU")
    from artis_amd import Engine
    from artis_amd.model import Model

    m = Model(ngrid_1d=args.ngrid)
    m.set_timestep(args.nts)
    eng = Engine(m, params=m.params)
    try:
        ms = []
        for u in range(args.uploads):
            eng.upload_cellstate(args.nts)
            ms.append(eng.last_precompute_ms())
            print(f"[precompute_ab] upload {u}: {ms[-1]:.1f} ms", file=sys.stderr, flush=True)
        print(json.dumps({"so": os.environ.get("ARTIS_GPU_SO", "in-tree"), "precompute_ms": ms,
                          "mean_ms": sum(ms[1:]) / max(1, len(ms) - 1), "tables": eng.table_info()}), flush=True)
    finally:
        eng.close()


if __name__ == "__main__":
    main()
