"""One nebular update_grid on the GPU (the free one-zone case of tests/test_gpu_nebular_update_grid.py, no oracle):
for rocprofv3 kernel statistics."""
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"),
                os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")]
import test_gpu_nebular_update_grid as T  # noqa: E402
from artis_amd import Engine  # noqa: E402

m, p, nt, arr, nts = T._onezone_case(int(sys.argv[1]) if len(sys.argv) > 1 else 12, pinned=False)
eng = Engine(m, params=p)
for rep in range(2):
    a = arr.copy()
    ms = eng.update_grid_nlte(nt, a)
    print(f"update_grid_nlte: {ms:.1f} ms, passes {a.iters[arr.mgi_list]}, T_e {a.Te[arr.mgi_list]}", flush=True)
eng.close()
