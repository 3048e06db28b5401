"""Committed golden vectors (tests/golden/*.npz, made by tests/golden/make_golden.py).

CPU: the synthetic-model generator reproduces the recorded inputs and the oracle reproduces the recorded
outputs bit for bit.  GPU: the HIP engine, driven through the C-ABI, reproduces the same outputs within the
parity tolerances of tests/parity.py.  (Regression vectors of the oracle; parity with the reference itself is
unpinned -- see make_golden.py.)
"""
import json
import os

import numpy as np
import pytest

import parity
from artis_amd import ffi

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CASES = ["grid3d", "shells1d", "sphere1d"]


def _load(name):
    z = np.load(os.path.join(GOLDEN, f"{name}.npz"))
    case = json.loads(bytes(z["meta"]).decode())
    return z, case


def _model(case):
    from artis_amd.model import Model

    return Model(**case["cfg"])


@pytest.mark.parametrize("name", CASES)
def test_oracle_reproduces_golden(name):
    import oracle_lib

    z, case = _load(name)
    m = _model(case)
    pk = None
    for nts in case["nts"]:
        m.set_timestep(nts)
        if pk is None:
            pk = m.init_rpackets(nts, case["npkts"], seed=case["seed"])
            assert pk.view(np.uint8).tobytes() == z["packets_in"].tobytes(), "model generator drifted"
        est, _ = oracle_lib.update_packets(m, nts, pk, nthreads=4)
    assert pk.view(np.uint8).tobytes() == z["packets_out"].tobytes()
    assert parity.counters_equal(est.counters, z["counters"])
    assert (est.ecounter == z["ecounter"]).all() and (est.acounter == z["acounter"]).all()
    assert np.allclose(est.J, z["J"], rtol=1e-12, atol=0)


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
def test_engine_reproduces_golden(name):
    from artis_amd import Engine

    z, case = _load(name)
    m = _model(case)
    pk = z["packets_in"].copy().view(ffi.PACKET_DTYPE)
    ref = z["packets_out"].copy().view(ffi.PACKET_DTYPE)
    eng = Engine(m)
    try:
        for nts in case["nts"]:
            m.set_timestep(nts)
            eng.upload_cellstate(nts)
            est = eng.update_packets(nts, pk)
    finally:
        eng.close()
    parity.assert_packets_match(pk, ref)
    assert parity.counters_equal(est.counters, z["counters"])
    assert (est.ecounter == z["ecounter"]).all() and (est.acounter == z["acounter"]).all()
    for f in ("J", "nuJ", "ffheating", "gamma", "bfheating"):
        y = z[f]
        assert np.abs(getattr(est, f) - y).max() <= parity.ESTIMATOR_RTOL * max(np.abs(y).max(), 1e-300), f
    assert est.struct.nesc == int(z["nesc"])
