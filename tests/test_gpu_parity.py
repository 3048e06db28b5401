"""HIP engine vs CPU oracle, through the C-ABI (libartis_gpu.so).  Needs an MI355X.

Every packet carries its own counter-based RNG stream (deviation D1), so the engine and the oracle propagate
the SAME packet histories: integer/enum/index fields are compared exactly, floating-point fields within
tests/parity.py:FP_RTOL, estimators within ESTIMATOR_RTOL and their event counters exactly.

At the bench size (50^3 grid, ~9.4e4 lines) the oracle cannot run the whole ensemble in seconds, but packets do
not interact within a timestep, so the oracle re-runs a random subset of the very same packets (same packet
numbers -> same streams) and those must match the engine's results for them one for one.
"""
import os

import numpy as np
import pytest

import oracle_lib
import parity
from artis_amd import Engine, ffi

pytestmark = pytest.mark.gpu


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


def _pair(model, eng, nts, npkts, seed):
    model.set_timestep(nts)
    pk0 = model.init_rpackets(nts, npkts, seed=seed)
    eng.upload_cellstate(nts)
    pg = pk0.copy()
    eg = eng.update_packets(nts, pg)
    po = pk0.copy()
    eo, wo = oracle_lib.update_packets(model, nts, po, nthreads=16)
    return pk0, pg, eg, po, eo, wo


def test_grid3d_packets_and_estimators(small_model, engine_factory):
    eng = engine_factory(small_model)
    _, pg, eg, po, eo, wo = _pair(small_model, eng, 10, 4000, seed=3)
    nbad, worst = parity.assert_packets_match(pg, po)
    parity.assert_estimators_match(eg, eo)
    # same work on both sides (per-packet histories identical); WK_MA_TRANS counts transitions the engine
    # actually touched (binary-search probes with the macro-atom cache) rather than the oracle's linear scan
    wg = eng.last_work()
    keep = np.arange(len(wg)) != 9
    assert (wg[keep] == wo[keep]).all(), (wg, wo)
    assert parity.spectrum_l1(pg, po) < 1e-9


def test_shell_model(shell_model, engine_factory):
    eng = engine_factory(shell_model)
    _, pg, eg, po, eo, _ = _pair(shell_model, eng, 6, 3000, seed=4)
    parity.assert_packets_match(pg, po)
    parity.assert_estimators_match(eg, eo)


def test_multi_timestep_chain(small_model, engine_factory):
    """Packets carried over three timesteps (cell state re-uploaded each step as update_grid would)."""
    eng = engine_factory(small_model)
    small_model.set_timestep(12)
    pk = small_model.init_rpackets(12, 2000, seed=5)
    pg, po = pk.copy(), pk.copy()
    for nts in (12, 13, 14):
        small_model.set_timestep(nts)
        eng.upload_cellstate(nts)
        eg = eng.update_packets(nts, pg)
        eo, _ = oracle_lib.update_packets(small_model, nts, po, nthreads=16)
        parity.assert_packets_match(pg, po)
        parity.assert_estimators_match(eg, eo)


def test_without_macroatom_cache_is_identical(small_model, engine_factory, monkeypatch):
    """The HBM macro-atom cache (binary search over cumulative rates) picks exactly the linear-scan choice."""
    small_model.set_timestep(9)
    pk = small_model.init_rpackets(9, 2000, seed=6)
    eng = engine_factory(small_model)
    eng.upload_cellstate(9)
    a = pk.copy()
    eng.update_packets(9, a)
    eng.close()
    monkeypatch.setenv("ARTIS_GPU_NO_MACACHE", "1")
    eng2 = engine_factory(small_model)
    eng2.upload_cellstate(9)
    b = pk.copy()
    eng2.update_packets(9, b)
    assert not parity.discrete_mismatch(a, b).any()
    assert max(parity.fp_max_rel(a, b).values()) <= parity.FP_RTOL


@pytest.mark.parametrize("env", [{"ARTIS_GPU_NO_LINECOEF": "1"}, {"ARTIS_GPU_LINECOEF_ROWS": "half"},
                                 {"ARTIS_GPU_MACACHE_ROWS": "half"},
                                 {"ARTIS_GPU_MACACHE_ROWS": "half", "ARTIS_GPU_MA_BUILD_SMALL": "0"},
                                 {"ARTIS_GPU_MACACHE_ROWS": "half", "ARTIS_GPU_MA_BUILD_SMALL": "64"},
                                 {"ARTIS_GPU_LINECOEF_ROWS": "1", "ARTIS_GPU_MACACHE_ROWS": "1"},
                                 {"ARTIS_GPU_NO_MACACHE": "1"}, {"ARTIS_GPU_LINECOEF_GATHER": "1"},
                                 {"ARTIS_GPU_LINECOEF_GATHER": "1", "ARTIS_GPU_LINECOEF_ROWS": "half"}],
                         ids=["no_linecoef", "half_linecoef", "half_macache", "half_macache_large_builds",
                              "half_macache_mixed_builds", "one_row_each", "no_macache", "linecoef_gather_kernel",
                              "half_linecoef_gather_kernel"])
def test_table_budgets_match_oracle(small_model, engine_factory, monkeypatch, env):
    """Per-cell tables that only fit the HBM budget for some cells -- line coefficients centre outwards, macro-atom
    key records per (cell, level) in level mode, built by the small-level and the large-level launch
    (ARTIS_GPU_MA_BUILD_SMALL moves the split); the line coefficients also by the gather kernel that
    k_linecoef_lds replaced (ARTIS_GPU_LINECOEF_GATHER) -- or for none (no line coefficients; an empty record pool: every
    macro-atom jump made by the whole wave from the exact sums, ma_coop_select) give the same packet histories as
    the oracle and the full-table engine."""
    small_model.set_timestep(11)
    pk = small_model.init_rpackets(11, 4000, seed=12)
    probe = engine_factory(small_model)
    full = probe.table_info()
    probe.close()
    assert full["linecoef_rows"] == full["cells"] and full["macache_rows"] == full["cells"]
    for k, v in env.items():
        monkeypatch.setenv(k, str(full["cells"] // 2) if v == "half" else v)
    eng = engine_factory(small_model)
    info = eng.table_info()
    if "ARTIS_GPU_NO_LINECOEF" in env:
        assert info["linecoef_rows"] == 0 and info["linecoef_bytes"] == 0
    if "ARTIS_GPU_LINECOEF_ROWS" in env:
        assert 0 < info["linecoef_rows"] < info["cells"]
    if "ARTIS_GPU_MACACHE_ROWS" in env or "ARTIS_GPU_NO_MACACHE" in env:
        assert info["macache_rows"] == 0 and info["ma_pool_bytes"] > 0 and info["marates_bytes"] > 0
    eng.upload_cellstate(11)
    if "ARTIS_GPU_MACACHE_ROWS" in env:
        assert eng.table_info()["ma_level_records"] > 0
    if "ARTIS_GPU_NO_MACACHE" in env:
        assert eng.table_info()["ma_level_records"] == 0
    pg, po = pk.copy(), pk.copy()
    eg = eng.update_packets(11, pg)
    eo, wo = oracle_lib.update_packets(small_model, 11, po, nthreads=16)
    parity.assert_packets_match(pg, po)
    parity.assert_estimators_match(eg, eo)
    wg = eng.last_work()
    keep = np.arange(len(wg)) != 9
    assert (wg[keep] == wo[keep]).all(), (wg, wo)


def test_partial_macroatom_cache_replaced_between_timesteps(small_model, engine_factory, monkeypatch):
    """Level mode with a pool of a third of the rows: each upload_cellstate places the (cell, level) records on the
    pairs the walks used most since the last placement; three chained timesteps stay on the oracle's histories, and
    after the first re-placement most sampled jumps fall on pairs with a record."""
    probe = engine_factory(small_model)
    ncells = probe.table_info()["cells"]
    probe.close()
    monkeypatch.setenv("ARTIS_GPU_MACACHE_ROWS", str(ncells // 3))
    eng = engine_factory(small_model)
    assert eng.table_info()["macache_rows"] == 0
    small_model.set_timestep(12)
    pk = small_model.init_rpackets(12, 3000, seed=13)
    pg, po = pk.copy(), pk.copy()
    for nts in (12, 13, 14):
        small_model.set_timestep(nts)
        eng.upload_cellstate(nts)
        eg = eng.update_packets(nts, pg)
        eo, _ = oracle_lib.update_packets(small_model, nts, po, nthreads=16)
        parity.assert_packets_match(pg, po)
        parity.assert_estimators_match(eg, eo)
    info = eng.table_info()
    assert info["ma_level_records"] > 0 and info["ma_jumps"] > 0
    assert info["ma_jumps_recorded"] >= 0.5 * info["ma_jumps"], info


def test_macroatom_records_in_many_batches_are_identical(small_model, engine_factory, monkeypatch):
    """k_marates writes the records in level batches through a scratch (k_marec transposes them); a scratch
    of one level's records forces one batch per level and must give the same packets."""
    small_model.set_timestep(9)
    pk = small_model.init_rpackets(9, 2000, seed=6)
    eng = engine_factory(small_model)
    eng.upload_cellstate(9)
    a = pk.copy()
    eng.update_packets(9, a)
    eng.close()
    monkeypatch.setenv("ARTIS_GPU_MAREC_SCRATCH_MB", "0")
    eng2 = engine_factory(small_model)
    eng2.upload_cellstate(9)
    b = pk.copy()
    eng2.update_packets(9, b)
    assert a.tobytes() == b.tobytes()


def test_resident_path_matches_host_path(small_model, engine_factory):
    """upload + update_packets_resident + download == update_packets, and snapshot/restore replays exactly."""
    eng = engine_factory(small_model)
    small_model.set_timestep(8)
    pk = small_model.init_rpackets(8, 3000, seed=8)
    eng.upload_cellstate(8)
    a = pk.copy()
    ea = eng.update_packets(8, a)
    eng.upload(pk)
    eng.snapshot()
    outs = []
    for _ in range(2):
        eng.restore()
        eng.zero_estimators()
        eng.step_resident(8)
        b = np.zeros_like(pk)
        eng.download(b)
        outs.append((b, eng.download_estimators()))
    for b, eb in outs:
        assert b.tobytes() == a.tobytes()
        assert (eb.counters == ea.counters).all()
        assert np.allclose(eb.J, ea.J, rtol=parity.ESTIMATOR_RTOL, atol=0)


def test_edge_cases(small_model, engine_factory):
    eng = engine_factory(small_model)
    nts = 7
    small_model.set_timestep(nts)
    eng.upload_cellstate(nts)
    # empty batch
    empty = np.zeros(0, dtype=ffi.PACKET_DTYPE)
    e = eng.update_packets(nts, empty)
    assert e.struct.nesc == 0 and e.J.sum() == 0
    # escaped packets and packets already at the end of the step are left untouched
    pk = small_model.init_rpackets(nts, 512, seed=9)
    pk["type"][::3] = ffi.TYPE_ESCAPE
    t2 = pk["prop_time"].max()
    po = pk.copy()
    oracle_lib.update_packets(small_model, nts, po, nthreads=16)
    done = po["prop_time"].max()
    pk["prop_time"][1::3] = done
    po = pk.copy()
    pg = pk.copy()
    eo, _ = oracle_lib.update_packets(small_model, nts, po, nthreads=16)
    eg = eng.update_packets(nts, pg)
    assert pg[::3].tobytes() == pk[::3].tobytes()
    assert pg[1::3].tobytes() == pk[1::3].tobytes()
    parity.assert_packets_match(pg, po)
    parity.assert_estimators_match(eg, eo)
    assert done >= t2
    # a single packet
    one = small_model.init_rpackets(nts, 1, seed=10)
    o1 = one.copy()
    eng.update_packets(nts, one)
    oracle_lib.update_packets(small_model, nts, o1, nthreads=1)
    parity.assert_packets_match(one, o1)
    # bad arguments fail loudly
    with pytest.raises(Exception):
        eng.update_packets(nts + 10**6, pk.copy())


def test_bench_size_subset_parity(engine_factory):
    """Full bench model (50^3 cells, 3 elements x 4 ions x ~300 levels, ~9.4e4 lines): 2e5 packets on the
    engine; 1500 randomly chosen of them re-run on the oracle must match one for one, with no discrete mismatch
    (rounds 3-5 allowed one; tools/mismatch_probe.py on this sample and the two below found none, so it is gone)."""
    from artis_amd.model import Model

    m = Model()
    nts = 10
    m.set_timestep(nts)
    P = 200_000
    pk0 = m.init_rpackets(nts, P, seed=11)
    eng = engine_factory(m)
    eng.upload_cellstate(nts)
    pg = pk0.copy()
    eg = eng.update_packets(nts, pg)
    rng = np.random.default_rng(0)
    idx = np.sort(rng.choice(P, size=1500, replace=False))
    po = pk0[idx].copy()
    oracle_lib.update_packets(m, nts, po, nthreads=16)
    parity.assert_packets_match(pg[idx], po)
    # size-independent properties of the whole ensemble
    esc = pg["type"] == ffi.TYPE_ESCAPE
    assert eg.struct.nesc == esc.sum()
    assert np.all(pg["prop_time"][~esc] == pg["prop_time"][~esc].max())
    assert np.isclose(eg.struct.cmf_lum, pg["e_cmf"][esc].sum(), rtol=1e-9)
    c = eg.counters
    assert c[0] + c[1] + c[4] + c[5] == c[7] + c[8] + c[9] + c[10]
    assert c[19] + c[20] + c[7] + c[8] == c[14] + c[15] + c[16] + c[17] + c[18]
    assert np.allclose(np.linalg.norm(pg["dir"], axis=1), 1.0, atol=1e-10)


def test_event_queue_engine_matches_megakernel(small_model, engine_factory, monkeypatch):
    """The event-queue kernels (wavefront.h) and the one-kernel path draw the same streams: identical packets."""
    small_model.set_timestep(11)
    pk = small_model.init_rpackets(11, 3000, seed=12)
    eng = engine_factory(small_model)
    eng.upload_cellstate(11)
    a = pk.copy()
    ea = eng.update_packets(11, a)
    assert eng.last_rounds() > 0
    wa = eng.last_work()
    eng.close()
    monkeypatch.setenv("ARTIS_GPU_ENGINE", "mega")
    eng2 = engine_factory(small_model)
    eng2.upload_cellstate(11)
    b = pk.copy()
    eb = eng2.update_packets(11, b)
    assert eng2.last_rounds() == 0
    assert a.tobytes() == b.tobytes()
    assert (ea.counters == eb.counters).all()
    assert (wa == eng2.last_work()).all()
    parity.assert_estimators_match(ea, eb)


def test_bf_and_kpacket_heavy_model(engine_factory):
    """Dense, low-ionisation-potential model: bf absorptions activate macro-atoms and k-packets, fb
    deactivations emit through select_continuum_nu, k-packets cool through every channel.  These rare paths
    run through the cold-call machinery of the r-packet kernel (a bug there once wrote stale cold words)."""
    from artis_amd.model import Model

    m = Model(ngrid_1d=6, nlevels_per_ion=30, n_ionising=30, max_lines=2000, ntstep=30, ionpot_scale=0.35,
              mass_msun=0.1, T0=8000.0)
    eng = engine_factory(m)
    _, pg, eg, po, eo, _ = _pair(m, eng, 10, 300, seed=3)
    c = eo.counters
    assert c[5] > 0 and c[10] > 0 and c[20] > 0, c  # bf activations, fb deactivations, k-packets from bf
    parity.assert_packets_match(pg, po)
    parity.assert_estimators_match(eg, eo)


def test_allocation_failures_fail_cleanly(small_model, engine_factory, monkeypatch):
    """An out-of-memory packet store, spectrum scratch or snapshot returns an error (no dangling pointers): with
    the injected limit removed the same engine runs normally and finalizes once (engine.hip alloc_packets,
    artis_gpu_spectrum)."""
    from artis_amd import EngineError

    eng = engine_factory(small_model)
    small_model.set_timestep(10)
    eng.upload_cellstate(10)
    pk = small_model.init_rpackets(10, 2000, seed=61)
    monkeypatch.setenv("ARTIS_GPU_FAIL_ALLOC_ABOVE", "4096")
    with pytest.raises(EngineError):
        eng.update_packets(10, pk.copy())
    with pytest.raises(EngineError):
        eng.spectrum()
    monkeypatch.delenv("ARTIS_GPU_FAIL_ALLOC_ABOVE")
    eng.upload(pk)
    monkeypatch.setenv("ARTIS_GPU_FAIL_ALLOC_ABOVE", "4096")
    with pytest.raises(EngineError):
        eng.snapshot()
    monkeypatch.delenv("ARTIS_GPU_FAIL_ALLOC_ABOVE")
    pg = pk.copy()
    eg = eng.update_packets(10, pg)
    po = pk.copy()
    eo, _ = oracle_lib.update_packets(small_model, 10, po, nthreads=16)
    parity.assert_packets_match(pg, po)
    parity.assert_estimators_match(eg, eo)
    spec, lc, _ = eng.spectrum()
    assert lc.sum() > 0
    eng.close()
    eng.close()  # idempotent


def test_estimator_block_roundtrip_and_rccl(small_model, engine_factory):
    """The device block (artis_gpu_estimator_block_to_device) equals the host pack of the downloaded estimators
    (artis_estimator_block_pack, what the gloo test reduces); a block written back (from_device) is what the next
    download returns; a one-rank RCCL communicator all-reduces it unchanged (artis_gpu_estimators_allreduce).
    The device buffer comes from the engine's own HIP runtime (libamdhip64.so.7, loaded by libartis_gpu.so)."""
    import ctypes as C

    from artis_amd import comm_unique_id, dist as adist

    eng = engine_factory(small_model)
    hip = C.CDLL("libamdhip64.so.7")
    small_model.set_timestep(10)
    eng.upload_cellstate(10)
    pk = small_model.init_rpackets(10, 2000, seed=62)
    eng.upload(pk)
    eng.zero_estimators()
    eng.step_resident(10)
    host = eng.download_estimators()
    hb = adist.pack_estimators(host)
    n = eng.estimator_block_doubles()
    assert n == len(hb)
    dptr = C.c_void_p()
    assert hip.hipMalloc(C.byref(dptr), C.c_size_t(8 * n)) == 0
    try:
        eng.estimator_block_to_device(dptr.value)
        db = np.zeros(n)
        assert hip.hipMemcpy(C.c_void_p(db.ctypes.data), dptr, C.c_size_t(8 * n), 2) == 0  # D2H
        assert np.array_equal(db, hb)
        db *= 2.0
        assert hip.hipMemcpy(dptr, C.c_void_p(db.ctypes.data), C.c_size_t(8 * n), 1) == 0  # H2D
        eng.estimator_block_from_device(dptr.value)
    finally:
        hip.hipFree(dptr)
    twice = eng.download_estimators()
    assert np.array_equal(adist.pack_estimators(twice), 2 * hb)
    eng.comm_init(0, 1, comm_unique_id())
    eng.allreduce_estimators()
    again = eng.download_estimators()
    assert np.array_equal(adist.pack_estimators(again), 2 * hb)


@pytest.mark.parametrize("rlc", [1, 2])
def test_rlc_emiss_rpkt_vs_oracle(small_model, engine_factory, rlc):
    """do_rlc_est 1 / 2 (input.txt line 9 = 2 / 3, input.cc:1976-1979): rlc_emiss_rpkt (grey_emissivities.cc:79-122)
    on every r-packet segment; rpkt_emiss compared with the oracle, packets unchanged by the estimator."""
    p = ffi.RunParams.from_buffer_copy(small_model.params)
    p.do_rlc_est = rlc
    eng = engine_factory(small_model, params=p)
    small_model.set_timestep(9)
    pk0 = small_model.init_rpackets(9, 3000, seed=17)
    eng.upload_cellstate(9)
    pg = pk0.copy()
    eg = eng.update_packets(9, pg)
    po = pk0.copy()
    eo, _ = oracle_lib.update_packets(small_model, 9, po, nthreads=16, params=p)
    parity.assert_packets_match(pg, po)
    parity.assert_estimators_match(eg, eo)
    assert (eo.rpkt_emiss > 0).sum() > 5


@pytest.mark.parametrize("walk", ["1", "0"])
def test_bounded_line_walk_matches_oracle(shell_model, small_model, engine_factory, monkeypatch, walk):
    """k_rpkt's bounded line walk (ARTIS_GPU_RPKT_WALK=1: at most RPKT_WALK_LINES lines of get_event's walk per pass,
    the walk resumed next pass; chosen by default when the previous transport's steps scanned > 8 lines each) and the
    whole-step instance both give the oracle's histories."""
    monkeypatch.setenv("ARTIS_GPU_RPKT_WALK", walk)
    for m, nts, seed in ((shell_model, 6, 61), (small_model, 10, 62)):
        eng = engine_factory(m)
        _, pg, eg, po, eo, _ = _pair(m, eng, nts, 3000, seed=seed)
        parity.assert_packets_match(pg, po)
        parity.assert_estimators_match(eg, eo)


@pytest.fixture(scope="module")
def many_cell_model():
    """26^3 grid: 9 200 non-empty cells, more than the few-cell binning's MA_BIN_LDS (8 192), so the macro-atom queue
    takes the many-cell binning (the producers' bin counts and k_ma_scatter)."""
    from artis_amd.model import Model

    return Model(ngrid_1d=26, nlevels_per_ion=40, n_ionising=15, max_lines=4000, ntstep=30)


# the engine's A/B switches select fallback paths the default run never takes:
# gathered tickets instead of the producers' pre-tickets (MA_PRE), the per-packet deactivation side arrays instead of
# the F-queue records (MF_REC), the per-entry binning pass instead of the producers' bin counts (BIN_PUSH, many cells)
# and the device-atomic binning instead of the block-local LDS counts (MA_BIN_BLK, few cells)
FALLBACKS = [{"ARTIS_GPU_MA_PRE": "0"}, {"ARTIS_GPU_MF_REC": "0"}, {"ARTIS_GPU_BIN_PUSH": "0"},
             {"ARTIS_GPU_MA_BIN_BLK": "0"}, {"ARTIS_GPU_MA_PRE": "0", "ARTIS_GPU_MF_REC": "0", "ARTIS_GPU_BIN_PUSH": "0"}]


@pytest.mark.parametrize("cells", ["few", "many"])
@pytest.mark.parametrize("env", FALLBACKS, ids=lambda e: "+".join(k[9:] + "=" + v for k, v in e.items()))
def test_fallback_switches_match_oracle(small_model, many_cell_model, engine_factory, monkeypatch, cells, env):
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    m = small_model if cells == "few" else many_cell_model
    eng = engine_factory(m)
    _, pg, eg, po, eo, _ = _pair(m, eng, 10, 3000, seed=71)
    parity.assert_packets_match(pg, po)
    parity.assert_estimators_match(eg, eo)
    assert eo.counters[4] > 1000 and eo.counters[9] > 1000  # bound-bound activations and deactivations
