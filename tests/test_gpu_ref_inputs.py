"""The BASELINE configurations on the GPU: HIP engine vs CPU oracle on the reference's own run inputs.  Needs an
MI355X.

* classic (BASELINE config 1): tests/classicmode_inputfiles -- input-newrun.txt (seed, 50 log timesteps 3-30 d,
  thick cells above grey depth 8, k-packet diffusion), the 78-shell DDC10 model.txt and its abundances.txt,
  mapped onto the 100^3 cuboid of artisoptions_classic.h:12-14; excitation temperature T_J, dipole scattering.
* kilonova (BASELINE config 4): tests/kilonova_inputfiles -- the 25-shell model.txt.xz (v_max 0.48 c, custom
  nuclide columns), 10 timesteps 0.4-10 d, every cell grey for the first 5 timesteps (input line 20 "0.0 5");
  relativistic Doppler (artisoptions_kilonova_lte.h:203), excitation temperature T_e (:36), 50^3 grid.
* a 100-shell W7-like 1D model (BASELINE config 2) and the 50^3 grid with virtual packets + polarisation
  (config 5) at bench size, as subset parity.

The atomic data stay synthetic (the reference's atomicdata_feconi is a download); Fe/Co/Ni
take their mass fractions from abundances.txt.  Packets: integer/enum/index fields identical, FP within
parity.FP_RTOL, estimators within parity.ESTIMATOR_RTOL (tests/parity.py).
"""
import os

import numpy as np
import pytest

import oracle_lib
import parity
from artis_amd import Engine, ffi
from artis_amd.model import Model

pytestmark = pytest.mark.gpu

REF = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ref_inputs")
ATOMIC = dict(nlevels_per_ion=40, n_ionising=15, max_lines=4000)


def ref_model(name, **kw):
    d = os.path.join(REF, name)
    mf = os.path.join(d, "model.txt.xz" if os.path.exists(os.path.join(d, "model.txt.xz")) else "model.txt")
    return Model(files=(os.path.join(d, "input-newrun.txt"), mf, os.path.join(d, "abundances.txt")), **kw)


@pytest.fixture
def engine_factory():
    made = []

    def make(model, **kw):
        e = Engine(model, **kw)
        made.append(e)
        return e

    yield make
    for e in made:
        e.close()


def _chain(model, eng, pk, steps):
    pg, po = pk.copy(), pk.copy()
    out = []
    for nts in steps:
        model.set_timestep(nts)
        eng.upload_cellstate(nts)
        eg = eng.update_packets(nts, pg)
        eo, wo = oracle_lib.update_packets(model, nts, po, nthreads=16)
        parity.assert_packets_match(pg, po)
        parity.assert_estimators_match(eg, eo)
        out.append((eg, eo, eng.last_work(), wo))
    return pg, po, out


def test_classic_inputfiles(engine_factory):
    m = ref_model("classicmode", ngrid_1d=100, **ATOMIC)
    assert m.npts_model == 78 and m.cfg.ntstep == 50 and m.params.seed == 1281360349
    assert m.params.excitation_temperature == ffi.TEXC_TJ and m.params.pol_dipole == 1
    eng = engine_factory(m)
    # a reference run starts from pellets at tmin: decays, gamma transport, deposition, thick-cell grey r-packets
    pk = m.init_pellets(3000, seed=51)
    _, _, out = _chain(m, eng, pk, range(0, 3))
    assert out[0][1].counters[26] > 0  # thick-cell scatterings (ESCOUNTER, rpkt_event_thickcell)
    # later timesteps: line opacity, macro-atoms and k-packets in the thinner outer shells
    m.set_timestep(30)
    pr = m.init_rpackets(30, 4000, seed=52)
    _, _, out = _chain(m, eng, pr, range(30, 32))
    w = out[0][3]
    assert w[8] > 0 and w[10] > 0  # macro-atom jumps, k-packets


def test_kilonova_inputfiles(engine_factory):
    m = ref_model("kilonova", ngrid_1d=50, relativistic=1, excitation_te=1, **ATOMIC)
    assert m.npts_model == 25 and m.cfg.ntstep == 10 and m.params.relativistic_doppler == 1
    assert m.params.excitation_temperature == ffi.TEXC_TE
    eng = engine_factory(m)
    pk = m.init_pellets(3000, seed=53)
    _chain(m, eng, pk, range(0, 2))  # all cells grey (num_grey_timesteps 5)
    m.set_timestep(5)
    pr = m.init_rpackets(5, 3000, seed=54)
    _, _, out = _chain(m, eng, pr, range(5, 7))
    w = out[0][3]
    assert w[2] > 0 and w[8] > 0  # lines scanned, macro-atom jumps


def test_excitation_temperature_te_differs_from_tj(engine_factory):
    """LTEPOP_EXCITATIONTEMPERATURE (ltepop.cc:338): with T_J = 0.8 T_e the T_e and T_J runs both match the
    oracle and differ from each other (the switch reaches the level populations of the line opacities)."""
    res = []
    for te in (0, 1):
        m = Model(ngrid_1d=8, nlevels_per_ion=30, n_ionising=12, max_lines=3000, ntstep=20, tj_scale=0.8,
                  excitation_te=te)
        eng = engine_factory(m)
        m.set_timestep(8)
        pk = m.init_rpackets(8, 3000, seed=55)
        pg, _, out = _chain(m, eng, pk, [8])
        res.append((pg, out[0][0]))
        eng.close()
    assert res[0][0].tobytes() != res[1][0].tobytes()
    assert not np.array_equal(res[0][1].J, res[1][1].J)


def test_w7_like_100_shells_subset(engine_factory):
    """BASELINE config 2 shape: 100-shell 1D model on a 50^3 cuboid, full synthetic atomic data; 1e5 packets on
    the engine, 1000 of them re-run on the oracle must match one for one."""
    m = Model(ngrid_1d=50, nshells_1d=100)
    assert m.npts_model == 100
    nts = 10
    m.set_timestep(nts)
    P = 100_000
    pk0 = m.init_rpackets(nts, P, seed=56)
    eng = engine_factory(m)
    eng.upload_cellstate(nts)
    pg = pk0.copy()
    eg = eng.update_packets(nts, pg)
    idx = np.sort(np.random.default_rng(1).choice(P, size=1000, replace=False))
    po = pk0[idx].copy()
    oracle_lib.update_packets(m, nts, po, nthreads=16)
    parity.assert_packets_match(pg[idx], po)
    esc = pg["type"] == ffi.TYPE_ESCAPE
    assert eg.struct.nesc == esc.sum()
    assert np.isclose(eg.struct.cmf_lum, pg["e_cmf"][esc].sum(), rtol=1e-9)


def _full_atom_subset(engine_factory, m, nts, seed, P=100_000, nsub=1000):
    """P packets on the engine with the bench's full synthetic atom (3603 levels, 93 798 lines); nsub of them re-run
    on the oracle must match one for one (a); the same nsub on the engine alone: estimators and counters equal the
    oracle's (b) -- for few-cell models these are k_rpkt's per-block LDS estimator sums at the timed atom size."""
    m.set_timestep(nts)
    pk0 = m.init_rpackets(nts, P, seed=seed)
    eng = engine_factory(m)
    eng.upload_cellstate(nts)
    pg = pk0.copy()
    eg = eng.update_packets(nts, pg)
    esc = pg["type"] == ffi.TYPE_ESCAPE
    assert eg.struct.nesc == esc.sum()
    assert np.isclose(eg.struct.cmf_lum, pg["e_cmf"][esc].sum(), rtol=1e-9)
    idx = np.sort(np.random.default_rng(seed).choice(P, size=nsub, replace=False))
    po = pk0[idx].copy()
    eo, wo = oracle_lib.update_packets(m, nts, po, nthreads=16)
    parity.assert_packets_match(pg[idx], po)
    eng.close()  # one engine per process (the C ABI binds one device context)
    eng2 = engine_factory(m)
    eng2.upload_cellstate(nts)
    ps = pk0[idx].copy()
    es = eng2.update_packets(nts, ps)
    parity.assert_packets_match(ps, po)
    parity.assert_estimators_match(es, eo)
    return eo, wo


def test_nebularonezone_full_atom_subset(engine_factory):
    """BASELINE config 3 at the timed size: the nebularonezone inputs with the nebular options and the bench's full
    atom (bench.py baseline_configs), 1e5 packets on the engine, 1000 re-run on the oracle."""
    m = ref_model("nebularonezone", ngrid_1d=50, nebular=1)
    assert m.npts_model == 1 and m.nlevels_total == 3603
    eo, wo = _full_atom_subset(engine_factory, m, 6, seed=58)
    assert wo[8] > 0 and wo[5] > 0 and eo.radfield_count.sum() > 0  # macro-atom jumps, bf continua, bin estimators


def test_kilonova_full_atom_subset(engine_factory):
    """BASELINE config 4 at the timed atom size: the kilonova inputs (25 shells, relativistic, T_e excitation) with
    the bench's full atom, 1e5 packets on the engine, 1000 re-run on the oracle."""
    m = ref_model("kilonova", ngrid_1d=50, relativistic=1, excitation_te=1)
    assert m.npts_model == 25 and m.nlevels_total == 3603
    eo, wo = _full_atom_subset(engine_factory, m, 6, seed=59)
    assert wo[2] > 0 and wo[8] > 0


def test_grid50_vpkt_pol_subset(engine_factory):
    """BASELINE config 5 shape: 50^3 grid, virtual packets with polarisation (4 observers x 4 spectra) at a
    timestep inside the vspec window.  (a) 1e5 packets on the engine; 600 of them re-run on the oracle must
    match one for one; (b) the same 600 on the engine alone: the virtual-packet spectra vstokes_i/q/u and the
    counters equal the oracle's."""
    m = Model()
    nts = 30
    m.set_timestep(nts)
    P = 100_000
    pk0 = m.init_rpackets(nts, P, seed=57)
    vc = ffi.VpktConfig(nz_obs=(0.9, 0.3, -0.3, -0.9), phi_obs_deg=(0.0, 100.0, 200.0, 300.0),
                        exclude=(0.0, -1.0, -2.0, 26.0))
    eng = engine_factory(m)
    eng.vpkt_init(vc)
    eng.upload_cellstate(nts)
    pg = pk0.copy()
    eng.update_packets(nts, pg)
    vfull = eng.vpkt_download()
    assert vfull.counters()["nvpkt"] > 0 and np.abs(vfull.vstokes[0]).max() > 0
    idx = np.sort(np.random.default_rng(2).choice(P, size=600, replace=False))
    po = pk0[idx].copy()
    eo, vo, _ = oracle_lib.update_packets_vpkt(m, nts, po, vc, nthreads=16)
    parity.assert_packets_match(pg[idx], po)
    eng.close()  # one engine per process (the C ABI binds one device context)
    eng2 = engine_factory(m)
    eng2.vpkt_init(vc)
    eng2.upload_cellstate(nts)
    ps = pk0[idx].copy()
    es = eng2.update_packets(nts, ps)
    vs = eng2.vpkt_download()
    parity.assert_packets_match(ps, po)
    parity.assert_estimators_match(es, eo)
    assert vs.counters() == vo.counters()
    scale = max(np.abs(vo.vstokes).max(), 1e-300)
    assert np.abs(vs.vstokes - vo.vstokes).max() <= parity.ESTIMATOR_RTOL * scale
    assert np.abs(vo.vstokes[0]).max() > 0
