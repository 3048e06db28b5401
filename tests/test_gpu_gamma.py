"""Pellets, gamma rays, non-thermal leptons, grey thick cells and relativistic Doppler shifts: HIP engine vs the
CPU oracle, packet by packet (same per-packet RNG streams, deviation D1).  Needs an MI355X.

Every reference run starts from radioactive pellets at tmin (packet_init, packet.cc:59-149): they decay
(update_pellet, update_packets.cc:71-135) into gamma packets (pellet_gamma_decay, gammapkt.cc:255-313) that
Compton-scatter, photo-absorb or pair-produce (do_gamma, gammapkt.cc:533-700) into non-thermal leptons
(do_ntlepton, nonthermal.cc:1877) and then k-packets, or into positrons / electrons / alphas that deposit
(do_nonthermal_predeposit, update_packets.cc:16-69).  The tests drive that whole chain from timestep 0.
"""
import numpy as np
import pytest

import oracle_lib
import parity
from artis_amd import Engine, EngineError, ffi
from artis_amd.model import Model

pytestmark = pytest.mark.gpu

# dense enough for gamma rays to deposit a good share of their energy in the first timesteps
GAMMA_CFG = dict(ngrid_1d=8, nlevels_per_ion=30, n_ionising=12, max_lines=3000, ntstep=20, mass_msun=0.3,
                 n_kpktdiffusion_timesteps=1000, kpktdiffusion_timescale=0.001)


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
    """Advance the same ensemble on the engine and the oracle over `steps`, comparing after every timestep."""
    pg, po = pk.copy(), pk.copy()
    out = []
    for nts in steps:
        model.set_timestep(nts)
        eng.upload_cellstate(nts)
        eg = eng.update_packets(nts, pg)
        eo, _ = oracle_lib.update_packets(model, nts, po, nthreads=16)
        parity.assert_packets_match(pg, po)
        parity.assert_estimators_match(eg, eo)
        out.append((eg, eo))
    return pg, po, out


def test_pellets_from_tmin_match_oracle(engine_factory):
    m = Model(**GAMMA_CFG)
    eng = engine_factory(m)
    pk = m.init_pellets(3000, seed=21)
    pg, po, out = _chain(m, eng, pk, range(0, 6))
    eg0, _ = out[0]
    s = eg0.struct
    # the chain was exercised: decays, gamma deposition, lepton deposition, earlier decays as k-packets
    assert sum(e.struct.pellet_decays for e, _ in out) > 100
    assert sum(e.struct.gamma_dep for e, _ in out) > 0
    assert s.counters[25] > 0  # K_STAT_FROM_EARLIERDECAY (update_packets.cc:127)
    assert sum(e.counters[21] for e, _ in out) > 0  # NT_STAT_FROM_GAMMA
    assert sum(e.counters[24] for e, _ in out) > 0  # NT_STAT_TO_KPKT
    assert sum(e.rpkt_emiss.sum() for e, _ in out) > 0  # grey gamma heating estimator (do_rlc_est)
    esc = pg["type"] == ffi.TYPE_ESCAPE
    assert (pg["escape_type"][esc] == ffi.TYPE_GAMMA).any()
    assert (pg["escape_type"][esc] == ffi.TYPE_RPKT).any()


def test_noninstant_particle_deposition(engine_factory):
    m = Model(**GAMMA_CFG, instant_particle_deposition=0)
    eng = engine_factory(m)
    pk = m.init_pellets(2000, seed=22)
    _chain(m, eng, pk, range(0, 4))


def test_grey_thick_cells(engine_factory):
    """Cells above the grey optical-depth threshold scatter r-packets coherently (rpkt_event_thickcell,
    rpkt.cc:491-509) and convert k-packets by do_kpkt_bb (update_packets.cc:183)."""
    m = Model(**GAMMA_CFG, thick_tau=0.05)
    m.set_timestep(2)
    eng = engine_factory(m)
    pk = m.init_rpackets(2, 2000, seed=23)
    _, _, out = _chain(m, eng, pk, range(2, 4))
    assert out[0][1].counters[26] > 0  # ESCOUNTER from thick-cell scatterings
    pe = m.init_pellets(1500, seed=24)
    _chain(m, eng, pe, range(0, 3))


def test_relativistic_doppler(engine_factory):
    """USE_RELATIVISTIC_DOPPLER_SHIFT (kilonova options): relativistic line distances (rpkt.cc:130-135) and
    Doppler factors (vectors.h:94-97) at v up to 0.25 c."""
    m = Model(**GAMMA_CFG, relativistic=1, vmax=7.5e9)
    eng = engine_factory(m)
    m.set_timestep(4)
    pk = m.init_rpackets(4, 2000, seed=25)
    _chain(m, eng, pk, range(4, 6))
    pe = m.init_pellets(1500, seed=26)
    _chain(m, eng, pe, range(0, 3))


def test_pellet_path_event_queue_matches_megakernel(engine_factory, monkeypatch):
    m = Model(**GAMMA_CFG)
    pk = m.init_pellets(2000, seed=27)
    m.set_timestep(0)
    eng = engine_factory(m)
    eng.upload_cellstate(0)
    a = pk.copy()
    ea = eng.update_packets(0, a)
    eng.close()
    monkeypatch.setenv("ARTIS_GPU_ENGINE", "mega")
    eng2 = engine_factory(m)
    eng2.upload_cellstate(0)
    b = pk.copy()
    eb = eng2.update_packets(0, b)
    assert a.tobytes() == b.tobytes()
    assert (ea.counters == eb.counters).all()
    parity.assert_estimators_match(ea, eb)


def test_pellets_without_gamma_spectra_fail_loudly(engine_factory):
    m = Model(**GAMMA_CFG)
    pk = m.init_pellets(64, seed=28)
    m.gamma_spectra = None  # the engine is not given the line lists
    eng = engine_factory(m)
    m.set_timestep(0)
    eng.upload_cellstate(0)
    with pytest.raises(EngineError):
        eng.update_packets(0, pk.copy())


def test_compton_emissivity_estimators_match_oracle(engine_factory):
    """Gamma-ray light-curve mode (do_r_lc = 0) with the Compton / pair-production emissivity estimators
    (emissivities.cc:14-136) on: packets identical, compton_emiss within float rounding of the oracle's."""
    from test_oracle_gamma import compton_params

    m = Model(**GAMMA_CFG)
    p = compton_params(m, outside_window=True)
    eng = engine_factory(m, params=p)
    pk = m.init_pellets(3000, seed=42)
    pg, po = pk.copy(), pk.copy()
    filled = 0
    for nts in range(0, 4):
        m.set_timestep(nts)
        eng.upload_cellstate(nts)
        eg = eng.update_packets(nts, pg)
        eo, _ = oracle_lib.update_packets(m, nts, po, nthreads=16, params=p)
        parity.assert_packets_match(pg, po)
        parity.assert_estimators_match(eg, eo)
        filled += int((eo.compton_emiss > 0).sum())
    assert filled > 10
