"""update_grid's temperature / ionisation solution (artis_gpu_solve_temperatures) on the CPU
oracle: the restated GSL Brent root finder, calculate_populations and call_T_e_finder checked through the properties
the reference's solution satisfies.  CPU only; the GPU parity tests are in test_gpu_te_solver.py.

Parity unpinned for this row: the reference writes its solution only into estimators_*.out files of full runs with
the downloaded atomic dataset (no fixture holds one); the checks here are the solver's own defining relations.
"""
import ctypes as C

import numpy as np
import pytest

import oracle_lib
from artis_amd import ffi
from artis_amd.model import Model

DAY = 86400.0


@pytest.fixture(scope="module")
def te_model():
    m = Model(ngrid_1d=6, nlevels_per_ion=30, n_ionising=12, max_lines=3000, ntstep=20)
    m.set_timestep(5)
    return m


def solve(m, **kw):
    te = ffi.TeArrays(m, t_current=10 * DAY, **kw)
    old = te.copy()
    assert oracle_lib.solve_temperatures(m, te) == 0
    return te, old


def test_lte_branch_sets_te_to_tj_and_balances_charge(te_model):
    """thick == 1 (update_grid.cc:1106-1125): T_e = T_J, LTE (Saha) ratios; n_e is the Brent root of
    nne_solution_f (ltepop.cc:20-59) to its 1e-3 interval accuracy."""
    m = te_model
    te, _ = solve(m, lte_all=True)
    idx = te.mgi_list
    assert np.array_equal(te.Te[idx], te.TJ[idx])
    assert np.all(te.iters[idx] == 0)
    ni = m.nions_total
    hdr = ffi.AtomicHeader.from_address(m.atomic)
    nions = np.ctypeslib.as_array(ffi.C.cast(hdr.elem_nions, ffi.C.POINTER(ffi.C.c_int32)), (m.nelements,))
    for mgi in idx[:20]:
        # sum over ions of charge x ion population (groundlevelpop * partfunct / g0, g0 cancels in the ratio check)
        assert te.nne[mgi] > 0 and np.isfinite(te.nne[mgi])
        assert np.all(te.partfunct[mgi * ni:(mgi + 1) * ni] >= 1.0)  # U >= g0 >= 1
        assert te.totalcooling[mgi] > 0
        assert np.isclose(te.totalcooling[mgi], te.cooling_contrib_ion[mgi * ni:(mgi + 1) * ni].sum(), rtol=1e-12)
    assert int(nions.sum()) == ni


def test_thermal_balance_root_and_bounds(te_model):
    """call_T_e_finder (thermalbalance.cc:397-597): T_e in [MINTEMP, MAXTEMP] and within the damping window
    [T_old/2, 2 T_old]; cells with a bracketed root end with |heating - cooling| small against either side."""
    m = te_model
    te, old = solve(m, thick_frac=0.0)
    idx = te.mgi_list
    p = te.params
    assert np.all(te.Te[idx] >= p.T_min) and np.all(te.Te[idx] <= p.T_max)
    assert np.all(te.Te[idx] <= 2 * old.Te[idx] * (1 + 1e-6))
    assert np.all(te.Te[idx] >= 0.5 * old.Te[idx] * (1 - 1e-6))
    r = te.rates.reshape(-1, ffi.TE_NRATES)
    rooted = idx[(te.iters[idx] > 0) & (te.Te[idx] < 2 * old.Te[idx] * 0.999) & (te.Te[idx] > 0.5 * old.Te[idx] * 1.001)]
    assert len(rooted) >= 3
    for mgi in rooted:
        heat = r[mgi, 4:8].sum()
        cool = r[mgi, 0:4].sum()
        # the Brent interval is 1e-2 in T_e: heating - cooling at its end point is a fraction of either side
        assert abs(heat - cool) <= 0.5 * max(heat, cool), (mgi, heat, cool)
    none = idx[te.iters[idx] == -1]
    assert len(none) + len(rooted) <= len(idx)


def test_nebular_phi_uses_gamma_estimators(te_model):
    """Outside LTE, phi = Alpha_sp / (Gamma g0 / U) (ltepop.cc:167-217) and uppermost_ion stops at the first ion
    with a zero photoionisation estimator (update_grid.cc:1463-1480): ions above it keep MINPOP."""
    m = te_model
    te = ffi.TeArrays(m, t_current=10 * DAY, gamma_zero_frac=0.0)
    te.gamma[:] = 0.0  # every Gamma zero: uppermost ion 0 everywhere -> the neutral-only branch
    assert oracle_lib.solve_temperatures(m, te) == 0
    idx = te.mgi_list
    ni = m.nions_total
    minpop = m.params.minpop if m.params.minpop > 0 else 1e-30
    hdr = ffi.AtomicHeader.from_address(m.atomic)
    off = np.ctypeslib.as_array(ffi.C.cast(hdr.elem_uniqueionoffset, ffi.C.POINTER(ffi.C.c_int32)), (m.nelements,))
    for mgi in idx[:10]:
        gp = te.groundlevelpop[mgi * ni:(mgi + 1) * ni]
        pf = te.partfunct[mgi * ni:(mgi + 1) * ni]
        for e in range(m.nelements):
            # the neutral-only branch: every ion but the first of each element at MINPOP (ion populations)
            u = off[e]
            nxt = off[e + 1] if e + 1 < m.nelements else ni
            for ui in range(u + 1, nxt):
                assert gp[ui] * pf[ui] > 0  # MINPOP * g0 / U * U / g0 (float rounding)
                assert gp[ui] <= 10 * minpop
        assert te.nne[mgi] >= minpop * 0.999


def test_solver_is_deterministic_and_leaves_unlisted_cells(te_model):
    m = te_model
    te1, old = solve(m)
    te2, _ = solve(m)
    for k in ("Te", "nne", "nnetot", "groundlevelpop", "partfunct", "totalcooling", "cooling_contrib_ion", "rates",
              "iters"):
        assert np.array_equal(getattr(te1, k), getattr(te2, k)), k
    # one listed cell only: every other cell's arrays come back unchanged
    te = ffi.TeArrays(m, t_current=10 * DAY)
    te.mgi_list = te.mgi_list[:1]
    before = te.copy()
    assert oracle_lib.solve_temperatures(m, te) == 0
    other = np.ones(m.npts_model, bool)
    other[te.mgi_list] = False
    assert np.array_equal(te.Te[other], before.Te[other])


def test_gsl_abort_path_is_an_error(te_model):
    """A cell whose n_e bracket [0, rho/m_H] does not straddle zero is a GSL_ERROR in gsl_root_fsolver_set, i.e. the
    reference aborts (update_grid.cc:1561-1585): the restatement reports ARTIS_ERR_PACKET_FAULT instead of a value."""
    m = te_model
    te = ffi.TeArrays(m, t_current=10 * DAY, lte_all=True)
    bad = te.mgi_list[3]
    te.elem_meanweight.reshape(-1, m.nelements)[bad, :] = 1e-30  # n_element huge: f(rho/m_H) > 0 as well
    assert oracle_lib.solve_temperatures(m, te) == -5


def _prepared(m, seed=6, **kw):
    g = ffi.AtomicHeader.from_address(m.atomic)
    te = ffi.TeArrays(m, t_current=10 * DAY, **kw)
    prep = ffi.UgArrays(m, deltat=0.5 * DAY, tratmid=3.0, seed=seed)
    assert oracle_lib.prepare_temperatures(m, te, prep) == 0
    return te, prep, g


def test_prepare_lte_and_fit_branches(te_model):
    """update_grid.cc:1106-1150: grey / initial cells get T_R = T_J = get_T_J_from_J, W = 1, corrphotoionrenorm 1;
    the others the fitted T_J, T_R (clamped to [MINTEMP, MAXTEMP]), W = pi J / sigma / T_R^4 and normalised
    estimators."""
    m = te_model
    te, prep, hdr = _prepared(m, thick_frac=0.3)
    idx = te.mgi_list
    lte = te.thick[idx] == 1
    assert lte.any() and (~lte).any()
    a, b = idx[lte], idx[~lte]
    assert np.array_equal(prep.TR_out[a], prep.TJ_out[a]) and np.all(prep.W_out[a] == 1.0)
    nm = m.nelements * m.maxnions
    assert np.all(prep.renorm_out.reshape(-1, nm)[a] == 1.0)
    assert np.all((prep.TR_out[b] >= hdr.mintemp) & (prep.TR_out[b] <= hdr.maxtemp))
    assert np.all(prep.W_out[b] > 0)
    assert np.all(prep.ff_out[b] > 0) and np.all(prep.col_out[b] > 0)
    # the prepared block feeds the temperature solution
    te.TR, te.W, te.TJ = prep.TR_out.copy(), prep.W_out.copy(), prep.TJ_out.copy()
    te.ffheating, te.colheating = prep.ff_out.copy(), prep.col_out.copy()
    te.gamma, te.bfheating = prep.gamma_out.copy(), prep.bfheating_out.copy()
    assert oracle_lib.solve_temperatures(m, te) == 0
    assert np.all(np.isfinite(te.Te[idx]))


def test_prepare_nonfinite_renorm_is_fatal(te_model):
    """update_gamma_corrphotoionrenorm_bfheating_estimators aborts on a non-finite corrphotoionrenorm or bf-heating
    ratio (update_grid.cc:911-918, 959-965): W_old = 0 in a non-LTE cell is such a case, an LTE-branch cell is not."""
    m = te_model
    te = ffi.TeArrays(m, t_current=10 * DAY, seed=11)
    prep = ffi.UgArrays(m, deltat=0.5 * DAY, tratmid=3.0, seed=3)
    assert oracle_lib.prepare_temperatures(m, te, prep) == 0
    te.W[te.mgi_list[1]] = 0
    prep = ffi.UgArrays(m, deltat=0.5 * DAY, tratmid=3.0, seed=3)
    assert oracle_lib.prepare_temperatures(m, te, prep) == -5
    te.thick[te.mgi_list[1]] = 1
    prep = ffi.UgArrays(m, deltat=0.5 * DAY, tratmid=3.0, seed=3)
    assert oracle_lib.prepare_temperatures(m, te, prep) == 0


def test_timestep_loop_update_grid_wiring_on_oracle():
    """artis_amd.timestep.LteTimestepLoop.update_grid with the oracle standing in for the engine's two update_grid
    calls (CPU): the previous step's raw estimators go through the preparation and the temperature solution, and the
    solved state (T_e, n_e, radiation field, populations, cooling, renormalisation) lands in the model's cell state
    that the next upload_cellstate reads."""
    from artis_amd.timestep import LteTimestepLoop

    m = Model(ngrid_1d=6, nlevels_per_ion=20, n_ionising=8, max_lines=800, ntstep=20)

    class OracleEngine:
        def prepare_temperatures(self, te, prep):
            assert oracle_lib.prepare_temperatures(m, te, prep) == 0

        def solve_temperatures(self, te):
            assert oracle_lib.solve_temperatures(m, te) == 0
            return 0.

    loop = LteTimestepLoop(m, OracleEngine())
    m.set_timestep(8)
    pk = m.init_rpackets(8, 2000, seed=4, etot=loop.radiation_energy(8))
    est, _ = oracle_lib.update_packets(m, 8, pk, nthreads=8)
    loop.update_grid(9, est)
    te = loop.solution
    g = te.mgi_list
    # every cell went through call_T_e_finder (-1: no root in [MINTEMP, MAXTEMP], which the synthetic atom's line
    # cooling makes the common outcome; the reference then takes MINTEMP and damps against the previous T_e)
    assert len(g) > 10 and (te.iters[g] != 0).all() and np.isfinite(te.Te[g]).all() and (te.Te[g] > 0).all()
    cs = ffi.CellState.from_address(m.cellstate)
    Te = np.ctypeslib.as_array(C.cast(cs.Te, C.POINTER(C.c_float)), (m.npts_model,))
    TR = np.ctypeslib.as_array(C.cast(cs.TR, C.POINTER(C.c_float)), (m.npts_model,))
    assert np.array_equal(Te[g], te.Te[g]) and np.array_equal(TR[g], te.TR[g])
    # the prepared radiation field comes from this step's J / nuJ: T_R differs from the stand-in's
    m2 = Model(ngrid_1d=6, nlevels_per_ion=20, n_ionising=8, max_lines=800, ntstep=20)
    m2.set_timestep(9)
    TR2 = np.ctypeslib.as_array(C.cast(ffi.CellState.from_address(m2.cellstate).TR, C.POINTER(C.c_float)),
                                (m2.npts_model,))
    assert not np.allclose(TR[g], TR2[g])
