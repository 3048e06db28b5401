"""GRID_SPHERICAL1D on the GPU: the spherical branch of boundary_cross with get_shellcrossdist (boundary.cc:14-99,
101-330) and the spherical maxsdist (rpkt.cc:659-661, gammapkt.cc:551-553), HIP engine vs CPU oracle through the
C ABI.  Needs an MI355X.  Same bar as tests/test_gpu_parity.py: discrete packet state identical, FP fields within
parity.FP_RTOL, estimators within parity.ESTIMATOR_RTOL with exact event counts.  The grid's geometric properties are
checked on the CPU in tests/test_spherical.py."""
import os

import numpy as np
import pytest

import oracle_lib
import parity
from artis_amd import Engine, ffi
from artis_amd.model import Model

pytestmark = pytest.mark.gpu

SPH = dict(nshells_1d=40, grid_spherical=1, nlevels_per_ion=40, n_ionising=15, max_lines=4000, ntstep=30)
REF = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ref_inputs")


@pytest.fixture(scope="module")
def sph_model():
    return Model(**SPH)


def _pair(m, nts, pk, **kw):
    m.set_timestep(nts)
    eng = Engine(m, **kw)
    try:
        eng.upload_cellstate(nts)
        pg = pk.copy()
        eg = eng.update_packets(nts, pg)
    finally:
        eng.close()
    po = pk.copy()
    eo, _ = oracle_lib.update_packets(m, nts, po, nthreads=16, params=kw.get("params"))
    parity.assert_packets_match(pg, po)
    parity.assert_estimators_match(eg, eo)
    return pg, eg, po, eo


@pytest.mark.parametrize("nts", [4, 12])
def test_spherical_rpackets_match_oracle(sph_model, nts):
    sph_model.set_timestep(nts)
    pk = sph_model.init_rpackets(nts, 6000, seed=51 + nts)
    pg, eg, po, eo = _pair(sph_model, nts, pk)
    assert eo.counters[28] > 10 * len(pk) and eo.struct.nesc > 100  # shell crossings, escapes


@pytest.mark.parametrize("walk", ["1", "0"])
def test_spherical_line_walks(sph_model, monkeypatch, walk):
    """The bounded and the whole-step line walks of k_rpkt (ARTIS_GPU_RPKT_WALK) on the spherical grid."""
    monkeypatch.setenv("ARTIS_GPU_RPKT_WALK", walk)
    sph_model.set_timestep(8)
    _pair(sph_model, 8, sph_model.init_rpackets(8, 3000, seed=57))


def test_spherical_pellets_gamma(sph_model):
    """Pellets placed in shells, decays and gamma rays through the shells over three timesteps."""
    pe = sph_model.init_pellets(5000, seed=58)
    for nts in (0, 1, 2):
        pe, _, _, _ = _pair(sph_model, nts, pe)


def test_spherical_classic_inputs():
    """The classic 1D inputs (tests/classicmode_inputfiles model.txt, 78 shells) on the spherical grid."""
    d = os.path.join(REF, "classicmode")
    m = Model(files=(os.path.join(d, "input-newrun.txt"), os.path.join(d, "model.txt"), os.path.join(d, "abundances.txt")),
              grid_spherical=1, nlevels_per_ion=40, n_ionising=15, max_lines=4000)
    m.set_timestep(12)
    _pair(m, 12, m.init_rpackets(12, 4000, seed=59))


def test_spherical_vpkt_match_oracle(sph_model):
    """Virtual packets traced through the shells to the outer boundary (vpkt.cc:76-368 calls boundary_cross)."""
    nts = 20
    sph_model.set_timestep(nts)
    pk = sph_model.init_rpackets(nts, 2000, seed=60)
    vc = ffi.VpktConfig(nz_obs=(0.3, -0.7), phi_obs_deg=(10.0, 200.0), exclude=(0.0, -1.0, 26.0))
    eng = Engine(sph_model)
    try:
        eng.vpkt_init(vc)
        eng.upload_cellstate(nts)
        pg = pk.copy()
        eg = eng.update_packets(nts, pg)
        vg = eng.vpkt_download()
    finally:
        eng.close()
    po = pk.copy()
    eo, vo, _ = oracle_lib.update_packets_vpkt(sph_model, nts, po, vc, nthreads=16)
    parity.assert_packets_match(pg, po)
    parity.assert_estimators_match(eg, eo)
    assert vo.counters()["nvpkt"] > 500
    assert vg.counters() == vo.counters()
    for a, b in ((vg.vstokes, vo.vstokes), (vg.vgrid, vo.vgrid)):
        assert np.abs(a - b).max() <= parity.ESTIMATOR_RTOL * max(np.abs(b).max(), 1e-300)
