"""Nebular update_grid on the GPU without the oracle, for rocprofv3 kernel statistics and timing: the free one-zone
case of tests/test_gpu_nebular_update_grid.py ('onezone', default) or every cell of the 6-shell synthetic nebular
model at timestep 12 ('multi': 136 cells, each with its Spencer-Fano solution)."""
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"),
                os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")]
import test_gpu_nebular_update_grid as T  # noqa: E402
from artis_amd import Engine, ffi  # noqa: E402
from artis_amd.model import Model  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "onezone"
if which == "multi":
    m = Model(**T.NEB)
    nts = 12
    p = ffi.RunParams.from_buffer_copy(m.params)
    est = T._estimators(m, p, nts - 1, 8000, seed=8)
    m.set_timestep(nts)
    nt = ffi.NtDataHandle(m)
    arr = ffi.NlteArrays(m, nts, est=est, seed=12)
    arr.params.num_lte_timesteps = 2
else:
    m, p, nt, arr, nts = T._onezone_case(12, pinned=False)
eng = Engine(m, params=p)
for rep in range(2):
    a = arr.copy()
    ms = eng.update_grid_nlte(nt, a)
    print(f"{which}: update_grid_nlte {ms:.1f} ms for {len(arr.mgi_list)} cells, passes max "
          f"{a.iters[arr.mgi_list].max()}", flush=True)
eng.close()
