"""Virtual packets (VPKT_ON): HIP engine (spawn buffer + k_vpkt, artis_amd/csrc/engine/vpkt.h) vs the CPU oracle
restatement of vpkt.cc.  Needs an MI355X.

The real packets must match the oracle exactly as without virtual packets (they draw no random numbers); the
event counters -- including the cell crossings and escapes of virtual packets, which the reference's change_cell
counts -- and nvpkt / nvpkt_esc1-3 must be identical; the polarised spectra vstokes_i/q/u and the velocity-grid
map are float64 atomic sums, compared within parity.ESTIMATOR_RTOL of their largest entry.
"""
import numpy as np
import pytest

import oracle_lib
import parity
from artis_amd import Engine, ffi
from artis_amd.model import Model

pytestmark = pytest.mark.gpu

VCFG = dict(ngrid_1d=8, nlevels_per_ion=30, n_ionising=12, max_lines=3000, ntstep=20)
NTS = 14  # inside the vspec window [10 d, 30 d]


def _compare_vpkt(vg, vo):
    assert vg.counters() == vo.counters()
    for a, b in ((vg.vstokes, vo.vstokes), (vg.vgrid, vo.vgrid)):
        # (a population inversion can make a virtual packet's tau so negative that exp(-tau) overflows: the
        # reference's bins then hold inf, and the engine's must hold the same)
        fa, fb = np.isfinite(a), np.isfinite(b)
        assert np.array_equal(fa, fb) and np.array_equal(a[~fb], b[~fb], equal_nan=True)
        scale = max(np.abs(b[fb]).max(initial=0.0), 1e-300)
        assert np.abs(a[fb] - b[fb]).max(initial=0.0) <= parity.ESTIMATOR_RTOL * scale


def _run(m, nts, pk, vc, engine_env=None, monkeypatch=None, upload_first=False):
    if engine_env and monkeypatch:
        monkeypatch.setenv("ARTIS_GPU_ENGINE", engine_env)
    eng = Engine(m)
    try:
        if upload_first:  # the per-cell tables (and their negative-coefficient flag) before the vpkt parameters
            eng.upload_cellstate(nts)
            eng.vpkt_init(vc)
        else:
            eng.vpkt_init(vc)
            eng.upload_cellstate(nts)
        pg = pk.copy()
        eg = eng.update_packets(nts, pg)
        vg = eng.vpkt_download()
        stats = eng.vpkt_last_stats()
    finally:
        eng.close()
    return pg, eg, vg, stats


def test_vpkt_matches_oracle():
    m = Model(**VCFG)
    m.set_timestep(NTS)
    pk = m.init_rpackets(NTS, 3000, seed=41)
    vc = ffi.VpktConfig(nz_obs=(0.3, -0.7, 1.0), phi_obs_deg=(10.0, 200.0, 0.0), exclude=(0.0, -1.0, -2.0, 26.0),
                        vgrid=True, ny_vgrid=25, nz_vgrid=25, grid_ranges_angstrom=((3500.0, 6000.0), (6000.0, 9000.0)))
    pg, eg, vg, (ms, spawns, traces) = _run(m, NTS, pk, vc)
    po = pk.copy()
    eo, vo, _ = oracle_lib.update_packets_vpkt(m, NTS, po, vc, nthreads=16)
    parity.assert_packets_match(pg, po)
    parity.assert_estimators_match(eg, eo)
    _compare_vpkt(vg, vo)
    c = vo.counters()
    assert c["nvpkt"] > 1000 and c["nvpkt_esc3"] > 0
    assert traces == c["nvpkt"] and spawns > 0 and ms > 0
    assert vg.vgrid[0].sum() > 0


def test_vpkt_escat_polarisation_and_megakernel(monkeypatch):
    """Electron-scattering virtual packets (realtype 1: Stokes rotation in and out of the scattering plane,
    vpkt.cc:124-180) in an e-scattering-rich model; the event-queue engine and the megakernel agree bit for bit
    on the packets and on the integer counters."""
    m = Model(**VCFG, mass_msun=0.3)
    m.set_timestep(NTS)
    pk = m.init_rpackets(NTS, 2000, seed=42)
    vc = ffi.VpktConfig(nz_obs=(0.0, 0.6), phi_obs_deg=(90.0, 300.0), exclude=(0.0, -4.0), tau_max=30.0)
    pg, eg, vg, _ = _run(m, NTS, pk, vc)
    po = pk.copy()
    eo, vo, _ = oracle_lib.update_packets_vpkt(m, NTS, po, vc, nthreads=16)
    parity.assert_packets_match(pg, po)
    _compare_vpkt(vg, vo)
    if vo.counters()["nvpkt_esc1"] > 0:
        assert np.abs(vg.vstokes[1]).sum() > 0
    pm, em, vm, _ = _run(m, NTS, pk, vc, engine_env="mega", monkeypatch=monkeypatch)
    assert pm.tobytes() == pg.tobytes()
    assert vm.counters() == vg.counters()
    assert (em.counters == eg.counters).all()
    _compare_vpkt(vm, vg)


def test_vpkt_multi_timestep_accumulates():
    """vstokes accumulate over timesteps (the reference keeps them for the whole run, vpkt.cc:21-23); the per-
    timestep counters reset on request (sn3d.cc:621-624)."""
    m = Model(**VCFG)
    pk = m.init_rpackets(13, 1500, seed=43)
    vc = ffi.VpktConfig(nz_obs=(0.4,), phi_obs_deg=(60.0,))
    eng = Engine(m)
    try:
        eng.vpkt_init(vc)
        pg, po = pk.copy(), pk.copy()
        vo = ffi.VpktArrays(vc)
        vg = ffi.VpktArrays(vc)
        for nts in (13, 14, 15):
            m.set_timestep(nts)
            eng.upload_cellstate(nts)
            eng.update_packets(nts, pg)
            eng.vpkt_download(vg, reset_counters=True)
            eng.vpkt_zero()
            oracle_lib.update_packets_vpkt(m, nts, po, vc, vout=vo, nthreads=16)
            parity.assert_packets_match(pg, po)
        _compare_vpkt(vg, vo)
    finally:
        eng.close()


def test_vpkt_full_spawn_buffer_drains_and_matches_oracle(monkeypatch):
    """A spawn buffer far smaller than one round's spawns (2048 records, with the persistent grids shrunk to 2048
    lanes so the overflow records are 2048 too): every launch that fills it is traced, its overflow records moved
    to the front and the launch resumed where it stopped -- the packets, counters and spectra are the oracle's."""
    monkeypatch.setenv("ARTIS_GPU_WAVE_GRID", "8")
    m = Model(**VCFG)
    m.set_timestep(NTS)
    pk = m.init_rpackets(NTS, 40000, seed=44)
    vc = ffi.VpktConfig(nz_obs=(0.3, -0.5), phi_obs_deg=(0.0, 120.0), exclude=(0.0, -1.0), spawn_capacity=16)
    eng = Engine(m)
    try:
        eng.vpkt_init(vc)
        eng.upload_cellstate(NTS)
        pg = pk.copy()
        eg = eng.update_packets(NTS, pg)
        vg = eng.vpkt_download()
        drains = eng.vpkt_last_drains()
        _, spawns, traces = eng.vpkt_last_stats()
    finally:
        eng.close()
    po = pk.copy()
    eo, vo, _ = oracle_lib.update_packets_vpkt(m, NTS, po, vc, nthreads=16)
    parity.assert_packets_match(pg, po)
    parity.assert_estimators_match(eg, eo)
    _compare_vpkt(vg, vo)
    assert drains > 0 and spawns > 2 * 2048, (drains, spawns)
    assert traces == vo.counters()["nvpkt"]


def test_vpkt_megakernel_full_buffer_fails_loudly(monkeypatch):
    """The megakernel (ARTIS_GPU_ENGINE=mega) cannot park packets on a full spawn buffer: with a buffer far below
    one round's spawns it must end the launch with an error, never hang or drop virtual packets silently."""
    monkeypatch.setenv("ARTIS_GPU_WAVE_GRID", "8")
    monkeypatch.setenv("ARTIS_GPU_ENGINE", "mega")
    m = Model(**VCFG)
    m.set_timestep(NTS)
    pk = m.init_rpackets(NTS, 40000, seed=44)
    vc = ffi.VpktConfig(nz_obs=(0.3, -0.5), phi_obs_deg=(0.0, 120.0), spawn_capacity=16)
    eng = Engine(m)
    try:
        eng.vpkt_init(vc)
        eng.upload_cellstate(NTS)
        with pytest.raises(RuntimeError):
            eng.update_packets(NTS, pk.copy())
    finally:
        eng.close()


@pytest.mark.parametrize("upload_first", [False, True])
def test_vpkt_nlte_inverted_lines_match_oracle(upload_first):
    """Virtual packets through NLTE populations with population inversions (negative Sobolev coefficients: the only
    case in which a virtual packet's tau can fall again).  The reference kills a virtual packet at the first line
    after which every spectrum's tau exceeds tau_max (vpkt.cc:280-283); k_vpkt tests at window ends and before
    every negative-coefficient line -- the same kills, so the spectra and counters are the oracle's.  Both call
    orders: vpkt_init after upload_cellstate must keep the table's negative-coefficient flag."""
    neb = dict(ngrid_1d=6, nlevels_per_ion=30, n_ionising=10, max_lines=2000, ntstep=20, nebular=1,
               nlte_level_max=12, tmin_days=100., tmax_days=300., T0=6000., ionpot_scale=0.5, mass_msun=50.)
    m = Model(**neb)
    nts = 14
    m.set_timestep(nts)
    ninv, ntot = oracle_lib.inverted_lines(m, nts)
    assert ninv > 0.002 * ntot, (ninv, ntot)
    pk = m.init_rpackets(nts, 2000, seed=46)
    vc = ffi.VpktConfig(nz_obs=(0.3, -0.7), phi_obs_deg=(10.0, 200.0), exclude=(0.0, -1.0, 26.0), tmin_days=100.0,
                        tmax_days=300.0, lambda_min=1000.0, lambda_max=30000.0, tau_max=1.0)
    pg, eg, vg, _ = _run(m, nts, pk, vc, upload_first=upload_first)
    po = pk.copy()
    eo, vo, _ = oracle_lib.update_packets_vpkt(m, nts, po, vc, nthreads=16)
    parity.assert_packets_match(pg, po)
    parity.assert_estimators_match(eg, eo)
    _compare_vpkt(vg, vo)
    c = vo.counters()
    assert c["nvpkt"] > 500 and c["nvpkt"] > c["nvpkt_esc1"] + c["nvpkt_esc2"] + c["nvpkt_esc3"]  # (kills)


@pytest.mark.parametrize("env", [("ARTIS_GPU_NO_LINECOEF", "1"), ("ARTIS_VPKT_LCONLY", "0")])
def test_vpkt_general_kernel_matches_oracle(monkeypatch, env):
    """k_vpkt's general instantiation (population-gather line walk: cells without a coefficient row, or forced with
    ARTIS_VPKT_LCONLY=0) against the oracle; the default table-only kernel runs in the other tests."""
    monkeypatch.setenv(*env)
    m = Model(**VCFG)
    m.set_timestep(NTS)
    pk = m.init_rpackets(NTS, 2000, seed=45)
    vc = ffi.VpktConfig(nz_obs=(0.3, -0.7), phi_obs_deg=(10.0, 200.0), exclude=(0.0, -1.0, 26.0))
    pg, eg, vg, _ = _run(m, NTS, pk, vc)
    po = pk.copy()
    eo, vo, _ = oracle_lib.update_packets_vpkt(m, NTS, po, vc, nthreads=16)
    parity.assert_packets_match(pg, po)
    parity.assert_estimators_match(eg, eo)
    _compare_vpkt(vg, vo)
    assert vo.counters()["nvpkt"] > 500


def test_vpkt_bounded_line_walk_full_buffer(monkeypatch):
    """The bounded r-packet line walk (ARTIS_GPU_RPKT_WALK=1) with a spawn buffer that fills mid-launch: a packet is
    parked only between steps, never inside a walk, and the results are the oracle's."""
    monkeypatch.setenv("ARTIS_GPU_WAVE_GRID", "8")
    monkeypatch.setenv("ARTIS_GPU_RPKT_WALK", "1")
    m = Model(**VCFG)
    m.set_timestep(NTS)
    pk = m.init_rpackets(NTS, 20000, seed=45)
    vc = ffi.VpktConfig(nz_obs=(0.3,), phi_obs_deg=(0.0,), spawn_capacity=16)
    eng = Engine(m)
    try:
        eng.vpkt_init(vc)
        eng.upload_cellstate(NTS)
        pg = pk.copy()
        eg = eng.update_packets(NTS, pg)
        vg = eng.vpkt_download()
        drains = eng.vpkt_last_drains()
    finally:
        eng.close()
    po = pk.copy()
    eo, vo, _ = oracle_lib.update_packets_vpkt(m, NTS, po, vc, nthreads=16)
    parity.assert_packets_match(pg, po)
    parity.assert_estimators_match(eg, eo)
    _compare_vpkt(vg, vo)
    assert drains > 0
