"""Find and describe the packets whose discrete state differs between the engine and the oracle in the three
bench-size subset parity tests (tests/test_gpu_parity.py::test_bench_size_subset_parity,
tests/test_gpu_ref_inputs.py::test_w7_like_100_shells_subset, ::test_config5_vpkt_subset shape): the packet number,
every integer field on both sides, and the FP fields.  GPU box only; writes JSON to stdout."""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

import oracle_lib  # noqa: E402
import parity  # noqa: E402
from artis_amd import Engine, ffi  # noqa: E402
from artis_amd.model import Model  # noqa: E402


def describe(pg, po):
    bad = parity.discrete_mismatch(pg, po)
    out = []
    for i in np.nonzero(bad)[0]:
        rec = {"number": int(po["number"][i])}
        for f in parity.INT_FIELDS:
            a, b = pg[f][i], po[f][i]
            if a.dtype.names:
                a = {k: int(a[k]) for k in a.dtype.names}
                b = {k: int(b[k]) for k in b.dtype.names}
            else:
                a, b = np.asarray(a).tolist(), np.asarray(b).tolist()
            if a != b:
                rec[f] = {"gpu": a, "oracle": b}
        for f in ("prop_time", "nu_cmf", "nu_rf", "e_cmf", "pos", "dir", "em_time", "absorptionfreq"):
            rec[f] = {"gpu": np.asarray(pg[f][i]).tolist(), "oracle": np.asarray(po[f][i]).tolist()}
        out.append(rec)
    return out


def run(case, m, nts, P, seed, nsub, rng_seed, vc=None):
    m.set_timestep(nts)
    pk0 = m.init_rpackets(nts, P, seed=seed)
    eng = Engine(m)
    if vc is not None:
        eng.vpkt_init(vc)
    eng.upload_cellstate(nts)
    pg = pk0.copy()
    eng.update_packets(nts, pg)
    eng.close()
    idx = np.sort(np.random.default_rng(rng_seed).choice(P, size=nsub, replace=False))
    po = pk0[idx].copy()
    if vc is None:
        oracle_lib.update_packets(m, nts, po, nthreads=16)
    else:
        oracle_lib.update_packets_vpkt(m, nts, po, vc, nthreads=16)
    d = describe(pg[idx], po)
    print(json.dumps({"case": case, "sample": nsub, "mismatches": d}), flush=True)
    return pk0, idx, d


if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1500
    run("bench_subset", Model(), 10, 200_000, 11, n, 0)
    run("w7_100_shells", Model(ngrid_1d=50, nshells_1d=100), 10, 100_000, 56, n, 1)
    vc = ffi.VpktConfig(nz_obs=(0.9, 0.3, -0.3, -0.9), phi_obs_deg=(0.0, 100.0, 200.0, 300.0),
                        exclude=(0.0, -1.0, -2.0, 26.0))
    run("config5_vpkt", Model(), 30, 100_000, 57, min(n, 600), 2, vc=vc)
