"""The nebular options (artisoptions_nltenebular.h) on the GPU: HIP engine vs CPU oracle.  Needs an MI355X.

Covers NLTE + superlevel populations (ltepop.cc:349-415), the binned radiation field in the macro-atom rates and
the NO_LUT photoionisation integrals (radfield.cc:898-943, ratecoeff.cc:1159-1308, integrated on the GPU by
qag.h), the detailed bf-rate and bin estimators (radfield.cc:764-876), the bf-estimator override of the
photoionisation coefficients, the non-thermal ionisation macro-atom action and do_ntlepton with the
Spencer-Fano solution (macroatom.cc:139-146, 866-884, nonthermal.cc:1584-1990).  Packets: integer fields
identical, FP within parity.FP_RTOL; estimators within parity.ESTIMATOR_RTOL, bin counts exact.
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
NEB = dict(ngrid_1d=6, nlevels_per_ion=30, n_ionising=10, max_lines=2000, ntstep=20, nebular=1, nlte_level_max=12,
           tmin_days=100., tmax_days=300., T0=6000., ionpot_scale=0.5)


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


def _pair(model, eng, nts, pk):
    model.set_timestep(nts)
    eng.upload_cellstate(nts)
    pg, po = pk.copy(), pk.copy()
    eg = eng.update_packets(nts, pg)
    eo, wo = oracle_lib.update_packets(model, nts, po, nthreads=16)
    parity.assert_packets_match(pg, po)
    parity.assert_estimators_match(eg, eo)
    return pg, eg, eo, wo


@pytest.mark.parametrize("nts", [5, 14])
def test_nebular_rpackets(engine_factory, nts):
    m = Model(**NEB)
    eng = engine_factory(m)
    m.set_timestep(nts)
    pk = m.init_rpackets(nts, 4000, seed=61 + nts)
    pg, eg, eo, wo = _pair(m, eng, nts, pk)
    assert wo[8] > 0 and eo.radfield_count.sum() > 0
    if nts >= 13:
        assert eo.bfrate_raw.sum() > 0


def test_nebular_pellets_ntlepton(engine_factory):
    """Decays -> gamma / leptons -> do_ntlepton: non-thermal ionisation activations and the NT macro-atom action."""
    m = Model(**NEB)
    eng = engine_factory(m)
    pe = m.init_pellets(6000, seed=62)
    total = np.zeros(ffi.ARTIS_COUNTER_COUNT, dtype=np.int64)
    for nts in (0, 1):
        pe, eg, eo, _ = _pair(m, eng, nts, pe)  # the next timestep continues from the propagated ensemble
        total += eo.counters
    assert total[22] > 0 and total[3] == total[22]


def test_nebular_nt_action_uncached(engine_factory, monkeypatch):
    """The same physics through the uncached macro-atom walk (k_ma<false>): identical results; the NT ionisation
    action (INTERNALUPHIGHERNT) is taken."""
    monkeypatch.setenv("ARTIS_GPU_NO_MACACHE", "1")
    m = Model(**NEB)
    eng = engine_factory(m)
    m.set_timestep(14)
    pk = m.init_rpackets(14, 4000, seed=63)
    _, eg, eo, _ = _pair(m, eng, 14, pk)
    tot = eo.counters.copy()
    eng.close()
    monkeypatch.delenv("ARTIS_GPU_NO_MACACHE")
    eng2 = engine_factory(m)
    pk2 = m.init_rpackets(14, 4000, seed=64)
    _, eg2, eo2, _ = _pair(m, eng2, 14, pk2)
    assert tot[12] + eo2.counters[12] > 0  # CTR_MA_STAT_INTERNALUPHIGHERNT


def test_nebularonezone_inputfiles(engine_factory):
    """tests/nebularonezone_inputfiles (the reference's nebular CI model, one zone) with the nebular options."""
    d = os.path.join(REF, "nebularonezone")
    m = Model(files=(os.path.join(d, "input-newrun.txt"), os.path.join(d, "model.txt"),
                     os.path.join(d, "abundances.txt")), ngrid_1d=10, nlevels_per_ion=30, n_ionising=10,
              max_lines=2000, nebular=1, nlte_level_max=12, ionpot_scale=0.5)
    assert m.npts_model == 1
    eng = engine_factory(m)
    m.set_timestep(5)
    pk = m.init_rpackets(5, 3000, seed=65)
    _pair(m, eng, 5, pk)
    pe = m.init_pellets(3000, seed=66)
    _pair(m, eng, 0, pe)


@pytest.mark.parametrize("env", [{"ARTIS_GPU_RPKT_COOP": "0"}, {"ARTIS_GPU_RPKT_COOP": "0", "ARTIS_GPU_MA_PRE": "0",
                                                                   "ARTIS_GPU_MF_REC": "0"}])
def test_nebular_detailed_bf_fallbacks(engine_factory, monkeypatch, env):
    """The detailed-bf model's fallback paths: per-lane continuum sums in k_rpkt instead of the wave-cooperative
    instance (RPKT_COOP=0), gathered tickets and per-packet deactivation side arrays -- the oracle's results."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    m = Model(**NEB)
    eng = engine_factory(m)
    m.set_timestep(14)
    pk = m.init_rpackets(14, 3000, seed=66)
    _, eg, eo, _ = _pair(m, eng, 14, pk)
    assert eo.bfrate_raw.sum() > 0
