"""update_grid's temperature / ionisation solution on the GPU (artis_gpu_solve_temperatures, SURVEY.md §8(f)
row 4) against the CPU oracle's restatement (oracle_solve_temperatures).  Needs an MI355X.

Both sides run the reference's serial algorithm in its operation order (GSL Brent on T_e, calculate_populations with
its own Brent on n_e, calculate_cooling_rates, calculate_heating_rates).  The device's exp/log/pow differ from glibc
in the last ulp, so the bar is: Brent iteration counts identical and T_e, n_e, partition functions, ground-level
populations, cooling and heating rates within TE_RTOL relative in at least 99 % of cells; in every cell T_e within
the solver's own interval accuracy (TEMPERATURE_SOLVER_ACCURACY, a branch of the Brent iteration may flip on an ulp).
"""
import os

import numpy as np
import pytest

import oracle_lib
import parity
from artis_amd import Engine, ffi
from artis_amd.model import Model

pytestmark = pytest.mark.gpu

DAY = 86400.0
TE_RTOL = 1e-9
REF = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ref_inputs")


def rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return np.abs(a - b) / np.maximum(np.maximum(np.abs(a), np.abs(b)), 1e-300)


def compare(m, te_gpu, te_cpu, min_frac=0.99):
    idx = te_gpu.mgi_list
    ni = m.nions_total
    same_it = te_gpu.iters[idx] == te_cpu.iters[idx]
    te_ok = rel(te_gpu.Te[idx], te_cpu.Te[idx]) <= TE_RTOL
    good = same_it & te_ok
    assert good.mean() >= min_frac, (good.mean(), idx[~good][:10])
    # every cell: within the T_e solver's interval accuracy
    assert np.all(rel(te_gpu.Te[idx], te_cpu.Te[idx]) <= 2 * te_cpu.params.accuracy)
    g = idx[good]
    for name, w in (("nne", 1), ("nnetot", 1), ("totalcooling", 1), ("groundlevelpop", ni), ("partfunct", ni),
                    ("cooling_contrib_ion", ni), ("rates", ffi.TE_NRATES)):
        a = getattr(te_gpu, name).reshape(-1, w)[g]
        b = getattr(te_cpu, name).reshape(-1, w)[g]
        r = rel(a, b)
        assert r.max() <= 1e-6, (name, r.max())
    # the stored cooling rates feed the next transport's k-packet ion selection: evaluated with the reference's
    # expression term for term (not the Brent iterations' reordered form), so where T_e (a float) is identical they
    # agree to the device libm's last-ulp differences (measured ~1e-12)
    same = g[te_gpu.Te[g] == te_cpu.Te[g]]
    if len(same):
        for name, w in (("totalcooling", 1), ("cooling_contrib_ion", ni)):
            r = rel(getattr(te_gpu, name).reshape(-1, w)[same], getattr(te_cpu, name).reshape(-1, w)[same])
            assert r.max() <= 1e-10, (name, r.max())
    return good.mean(), int((te_gpu.iters[idx] > 0).sum())


def run_both(m, te, params=None, engine_params=None):
    cpu = te.copy()
    assert oracle_lib.solve_temperatures(m, cpu, params=params) == 0
    eng = Engine(m, params=engine_params if engine_params is not None else params)
    try:
        ms = eng.solve_temperatures(te)
    finally:
        eng.close()
    return te, cpu, ms


@pytest.fixture(scope="module")
def small():
    m = Model(ngrid_1d=8, nlevels_per_ion=40, n_ionising=15, max_lines=4000, ntstep=20)
    m.set_timestep(6)
    return m


@pytest.mark.parametrize("thick_frac", [0.0, 0.3])
def test_gpu_te_solver_matches_oracle(small, thick_frac):
    te = ffi.TeArrays(small, t_current=12 * DAY, thick_frac=thick_frac, seed=5)
    g, c, ms = run_both(small, te)
    frac, rooted = compare(small, g, c)
    assert rooted > 10
    print(f"cells {len(te.mgi_list)}, agreeing {frac:.3f}, rooted {rooted}, {ms:.2f} ms")


@pytest.mark.parametrize("lanes", ["16", "1"])
def test_gpu_te_solver_lane_groups(small, monkeypatch, lanes):
    """ARTIS_GPU_TE_LANES: 16 lanes per cell (the round-4 layout) and one cell per lane instead of one lane per ion --
    the per-ion sums and their exchange take other paths, the results do not change."""
    monkeypatch.setenv("ARTIS_GPU_TE_LANES", lanes)
    te = ffi.TeArrays(small, t_current=12 * DAY, thick_frac=0.3, seed=5)
    g, c, _ = run_both(small, te)
    compare(small, g, c)


def test_gpu_te_solver_excitation_te_and_initial_iteration(small):
    """LTEPOP_EXCITATIONTEMPERATURE = T_e (artisoptions_kilonova_lte.h:36): the level populations follow every trial
    T_e; and initial_iteration (every cell in the LTE branch, update_grid.cc:1106)."""
    p = ffi.RunParams.from_buffer_copy(small.params)
    p.excitation_temperature = 1
    te = ffi.TeArrays(small, t_current=12 * DAY, seed=9)
    g, c, _ = run_both(small, te, params=p)
    compare(small, g, c)
    te = ffi.TeArrays(small, t_current=12 * DAY, seed=9)
    te.params.initial_iteration = 1
    g, c, _ = run_both(small, te)
    compare(small, g, c, min_frac=1.0)
    assert np.array_equal(g.Te[g.mgi_list], g.TJ[g.mgi_list])


def test_gpu_te_solver_classic_inputs():
    """The classic run inputs (tests/classicmode_inputfiles: 78 shells, T_J excitation)."""
    d = os.path.join(REF, "classicmode")
    m = Model(files=(os.path.join(d, "input-newrun.txt"), os.path.join(d, "model.txt"), os.path.join(d, "abundances.txt")),
              nlevels_per_ion=40, n_ionising=15, max_lines=4000)
    m.set_timestep(12)
    te = ffi.TeArrays(m, t_current=m.cfg.tmin_days * DAY * 2, seed=2)
    g, c, _ = run_both(m, te)
    compare(m, g, c)


def test_gpu_te_solver_bench_grid_subset():
    """The 50^3 bench model: the GPU solves every non-empty cell, the oracle a 256-cell subset."""
    m = Model(ngrid_1d=50)
    m.set_timestep(10)
    te = ffi.TeArrays(m, t_current=15 * DAY, seed=4)
    eng = Engine(m)
    try:
        ms = eng.solve_temperatures(te)
    finally:
        eng.close()
    sub = ffi.TeArrays(m, t_current=15 * DAY, seed=4)
    rng = np.random.default_rng(0)
    sub.mgi_list = np.sort(rng.choice(sub.mgi_list, 256, replace=False)).astype(np.int32)
    assert oracle_lib.solve_temperatures(m, sub) == 0
    te.mgi_list = sub.mgi_list
    compare(m, te, sub)
    print(f"50^3: {len(ffi.TeArrays(m, t_current=15 * DAY).mgi_list)} cells solved in {ms:.1f} ms")


def test_gpu_te_solver_kilonova_inputs():
    """The kilonova run inputs (tests/kilonova_inputfiles: 25 shells, MINTEMP 500 K) with the T_e excitation
    temperature of artisoptions_kilonova_lte.h:36."""
    d = os.path.join(REF, "kilonova")
    m = Model(files=(os.path.join(d, "input-newrun.txt"), os.path.join(d, "model.txt.xz"),
                     os.path.join(d, "abundances.txt")), nlevels_per_ion=40, n_ionising=15, max_lines=4000)
    m.set_timestep(6)
    p = ffi.RunParams.from_buffer_copy(m.params)
    p.excitation_temperature = 1
    te = ffi.TeArrays(m, t_current=m.cfg.tmin_days * DAY * 3, seed=8)
    g, c, _ = run_both(m, te, params=p)
    compare(m, g, c)


def test_gpu_te_solver_gsl_abort_path(small):
    """The reference's abort path (an n_e bracket that does not straddle zero) comes back as ARTIS_ERR_PACKET_FAULT
    naming the model cell, on the device as in the oracle."""
    from artis_amd import EngineError

    te = ffi.TeArrays(small, t_current=12 * DAY, lte_all=True)
    bad = int(te.mgi_list[3])
    te.elem_meanweight.reshape(-1, small.nelements)[bad, :] = 1e-30
    assert oracle_lib.solve_temperatures(small, te.copy()) == -5
    eng = Engine(small)
    try:
        with pytest.raises(EngineError, match=f"model cell {bad}"):
            eng.solve_temperatures(te)
    finally:
        eng.close()


@pytest.mark.parametrize("thick_frac", [0.0, 0.3])
def test_gpu_prepare_temperatures_matches_oracle(small, thick_frac):
    """update_grid_cell's estimator preparation (artis_gpu_prepare_temperatures, update_grid.cc:1041-1150) against
    the oracle, then the temperature solution on the prepared block: float outputs within one float ulp, doubles
    within TE_RTOL (device exp/log/pow last-ulp differences)."""
    te = ffi.TeArrays(small, t_current=12 * DAY, thick_frac=thick_frac, seed=11)
    pg = ffi.UgArrays(small, deltat=0.5 * DAY, tratmid=3.0, seed=3)
    pc = ffi.UgArrays(small, deltat=0.5 * DAY, tratmid=3.0, seed=3)
    assert oracle_lib.prepare_temperatures(small, te, pc) == 0
    eng = Engine(small)
    try:
        eng.prepare_temperatures(te, pg)
        idx = te.mgi_list
        for k in ("TR_out", "W_out", "TJ_out"):
            a, b = getattr(pg, k)[idx], getattr(pc, k)[idx]
            assert np.all(rel(a, b) <= 2.5e-7), (k, rel(a, b).max())
        nm = small.nelements * small.maxnions
        for k, w in (("ff_out", 1), ("col_out", 1), ("gamma_out", nm), ("bfheating_out", nm), ("renorm_out", nm)):
            a, b = getattr(pg, k).reshape(-1, w)[idx], getattr(pc, k).reshape(-1, w)[idx]
            fin = np.isfinite(b)
            assert np.array_equal(np.isfinite(a), fin), k
            assert np.all(rel(a[fin], b[fin]) <= TE_RTOL), (k, rel(a[fin], b[fin]).max())
        # chained: the solution from the device-prepared inputs against the oracle's
        for t, p in ((te, pg),):
            t.TR, t.W, t.TJ = p.TR_out.copy(), p.W_out.copy(), p.TJ_out.copy()
            t.ffheating, t.colheating = p.ff_out.copy(), p.col_out.copy()
            t.gamma, t.bfheating = p.gamma_out.copy(), p.bfheating_out.copy()
        cpu = te.copy()
        assert oracle_lib.solve_temperatures(small, cpu) == 0
        eng.solve_temperatures(te)
    finally:
        eng.close()
    compare(small, te, cpu)


def test_gpu_prepare_temperatures_fatal_nonfinite(small):
    """W_old = 0 in one non-LTE cell makes corrphotoionrenorm = Gamma / (W LUT) infinite: the reference aborts
    (update_grid.cc:911-918); device and oracle return ARTIS_ERR_PACKET_FAULT naming the cell, and the device leaves
    the caller's outputs unwritten."""
    from artis_amd import EngineError

    te = ffi.TeArrays(small, t_current=12 * DAY, thick_frac=0.0, seed=11)
    bad = int(te.mgi_list[2])
    te.W[bad] = 0
    pc = ffi.UgArrays(small, deltat=0.5 * DAY, tratmid=3.0, seed=3)
    assert oracle_lib.prepare_temperatures(small, te, pc) == -5
    pg = ffi.UgArrays(small, deltat=0.5 * DAY, tratmid=3.0, seed=3)
    before = pg.TR_out.copy()
    eng = Engine(small)
    try:
        with pytest.raises(EngineError, match=f"model cell {bad}"):
            eng.prepare_temperatures(te, pg)
    finally:
        eng.close()
    assert np.array_equal(pg.TR_out, before)


def test_timestep_loop_on_device_matches_oracle():
    """sn3d.cc's do_timestep body with every per-timestep stage on the device (artis_amd.timestep.LteTimestepLoop):
    update_grid's preparation + temperature solution from the previous step's raw estimators, upload_cellstate and
    update_packets on resident packets, three consecutive timesteps.  Each update_grid against the oracle's replay
    of the same inputs; each transport step against the oracle on the solved cell state."""
    from artis_amd.timestep import LteTimestepLoop

    m = Model(ngrid_1d=8, nlevels_per_ion=30, n_ionising=12, max_lines=3000, ntstep=20)
    nts0 = 8
    m.set_timestep(nts0)
    eng = Engine(m)
    try:
        loop = LteTimestepLoop(m, eng, keep_inputs=True)
        pk0 = m.init_rpackets(nts0, 3000, seed=19, etot=loop.radiation_energy(nts0))
        eng.upload(pk0)
        po = pk0.copy()
        est = None
        for k in range(3):
            nts = nts0 + k
            if k > 0:
                loop.update_grid(nts, est)
                te_in, ug_in = loop.last_inputs
                assert oracle_lib.prepare_temperatures(m, te_in, ug_in) == 0
                te_in.TR, te_in.W, te_in.TJ = ug_in.TR_out, ug_in.W_out, ug_in.TJ_out
                te_in.ffheating, te_in.colheating = ug_in.ff_out, ug_in.col_out
                te_in.gamma, te_in.bfheating = ug_in.gamma_out, ug_in.bfheating_out
                assert oracle_lib.solve_temperatures(m, te_in) == 0
                gte, g = loop.solution, te_in.mgi_list
                agree = (gte.iters[g] == te_in.iters[g]) & (np.abs(gte.Te[g] - te_in.Te[g]) <= 1e-9 * te_in.Te[g])
                assert agree.mean() >= 0.99, agree.mean()
                assert (gte.iters[g] != 0).all()  # every cell through call_T_e_finder (no LTE branch)
            eng.upload_cellstate(nts)
            eng.zero_estimators()
            eng.step_resident(nts)
            est = eng.download_estimators()
            pg = np.zeros_like(pk0)
            eng.download(pg)
            eo, _ = oracle_lib.update_packets(m, nts, po, nthreads=16)
            parity.assert_packets_match(pg, po)
            parity.assert_estimators_match(est, eo)
    finally:
        eng.close()
