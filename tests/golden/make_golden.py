"""Regenerate tests/golden/*.npz: oracle outputs for small seeded synthetic models.

    python tests/golden/make_golden.py

These are REGRESSION vectors produced by the CPU oracle (oracle/oracle.cc), not reference outputs: the
reference cannot be built here (needs GSL, see DESIGN.md "Oracle") and ships no usable golden vectors
(SURVEY.md §8c), so parity with the reference itself is unpinned.  The vectors pin the oracle across
changes and give the GPU tests a fixed target.  Inputs are regenerated from the recorded model config and
packet seed by the deterministic synthetic-model generator (artis_amd/csrc/host/model_synth.cc).
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

CASES = {
    "grid3d": dict(cfg=dict(ngrid_1d=8, nlevels_per_ion=40, n_ionising=15, max_lines=3000, ntstep=30),
                   nts=[6, 7], npkts=256, seed=21),
    "shells1d": dict(cfg=dict(ngrid_1d=10, nshells_1d=10, nlevels_per_ion=30, n_ionising=12, max_lines=2000,
                              ntstep=30), nts=[4], npkts=256, seed=22),
    # GRID_SPHERICAL1D (round 6): the shells as radial propagation cells
    "sphere1d": dict(cfg=dict(nshells_1d=20, grid_spherical=1, nlevels_per_ion=30, n_ionising=12, max_lines=2000,
                              ntstep=30), nts=[4, 5], npkts=256, seed=23),
}


def run_case(case):
    import oracle_lib
    from artis_amd.model import Model

    m = Model(**case["cfg"])
    pk = None
    ests = []
    for k, nts in enumerate(case["nts"]):
        m.set_timestep(nts)
        if pk is None:
            pk = m.init_rpackets(nts, case["npkts"], seed=case["seed"])
            pk_in = pk.copy()
        est, _ = oracle_lib.update_packets(m, nts, pk, nthreads=1)
        ests.append(est)
    return m, pk_in, pk, ests


def main():
    for name, case in CASES.items():
        m, pk_in, pk_out, ests = run_case(case)
        e = ests[-1]
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), packets_in=pk_in.view(np.uint8),
                            packets_out=pk_out.view(np.uint8), J=e.J, nuJ=e.nuJ, ffheating=e.ffheating,
                            gamma=e.gamma, bfheating=e.bfheating, counters=e.counters, ecounter=e.ecounter,
                            acounter=e.acounter, nesc=np.int64(e.struct.nesc), cmf_lum=np.float64(e.struct.cmf_lum),
                            meta=np.frombuffer(json.dumps(case).encode(), dtype=np.uint8))
        print(name, "escaped", int((pk_out["type"] == 32).sum()), "of", len(pk_out))


if __name__ == "__main__":
    main()
