"""Dump and compare the first-pass NLTE matrices of the pinned one-zone case (tests/test_gpu_nebular_update_grid.py)
on the GPU box.  Diagnostics only."""
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"),
                os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")]
import test_gpu_nebular_update_grid as T  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import nl_dump_cmp  # noqa: E402

os.makedirs(os.path.join("gpurun_out", "nld"), exist_ok=True)
prefix = os.path.join("gpurun_out", "nld", "d")
for f in os.listdir(os.path.join("gpurun_out", "nld")):
    os.remove(os.path.join("gpurun_out", "nld", f))
os.environ["ARTIS_GPU_NL_DUMP"] = prefix
os.environ["ORACLE_NL_DUMP"] = prefix
m, p, nt, arr, nts = T._onezone_case(12, pinned=True)
arr.params.nlteiter = int(sys.argv[1]) if len(sys.argv) > 1 else 1
ao, ag, ms = T._solve_both(m, p, arr, nt)
print("gpu ms", ms, "Te", ag.Te[arr.mgi_list], ao.Te[arr.mgi_list], "nne", ag.nne[arr.mgi_list], ao.nne[arr.mgi_list])
rep = T._report(ao, ag)
print("max rel diff: " + ", ".join(f"{k} {v:.1e}" for k, v in rep.items() if v > 0))
nl_dump_cmp.main(prefix, 4)
