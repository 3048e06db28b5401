"""update_grid for the nebular options on the GPU (artis_gpu_update_grid_nlte, nlte_solver.h) against the oracle's
restatement (oracle/nebular_update_grid.cc).  Needs an MI355X.

Per listed cell: the radiation-field fits (radfield.cc:1136-1291), the NO_LUT bf-heating coefficients, the
Spencer-Fano solution and its analysis (nonthermal.cc:1996-2713), call_T_e_finder, the NLTE rate matrices with
their LU solve and refinement (nltepop.cc:421-1113), the convergence loop of solve_Te_nltepops
(update_grid.cc:763-886) and the cooling rates.  Both sides read the same raw estimators (a GPU transport step of
the same model).  Integer outputs (pass counts, solved-timestep marks, the -1 "no NLTE solution" markers) must be
identical; floating-point outputs agree to NEB_RTOL -- the two sides differ only by last-bit differences of the
device libm, amplified by the iterative solves (Brent, LU refinement), which is what this tolerance bounds.
"""
import os

import numpy as np
import pytest

import oracle_lib
from artis_amd import Engine, ffi
from artis_amd.model import Model

pytestmark = pytest.mark.gpu

REF = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ref_inputs", "nebularonezone")
ONEZONE = dict(ngrid_1d=10, nlevels_per_ion=30, n_ionising=10, max_lines=2000, nebular=1, nlte_level_max=12,
               ionpot_scale=0.5)
NEB = dict(ngrid_1d=6, nlevels_per_ion=30, n_ionising=10, max_lines=2000, ntstep=20, nebular=1, nlte_level_max=12,
           tmin_days=100., tmax_days=300., T0=6000., ionpot_scale=0.5)
NEB_RTOL = 1e-5  # relative; populations below POP_ATOL (cm^-3, of 1e-3..1e6 totals) compared absolutely
POP_ATOL = 1e-20


def _onezone():
    return Model(files=(os.path.join(REF, "input-newrun.txt"), os.path.join(REF, "model.txt"),
                        os.path.join(REF, "abundances.txt")), **ONEZONE)


def _estimators(model, params, nts_prev, npkts, seed):
    """The raw estimators of one GPU transport step at nts_prev."""
    eng = Engine(model, params=params)
    try:
        model.set_timestep(nts_prev)
        eng.upload_cellstate(nts_prev)
        pk = model.init_rpackets(nts_prev, npkts, seed=seed)
        return eng.update_packets(nts_prev, pk)
    finally:
        eng.close()


def _solve_both(model, params, arr, nt):
    """The same NlteArrays block through the oracle and the engine; returns (oracle, gpu, ms)."""
    ao, ag = arr.copy(), arr.copy()
    rc = oracle_lib.update_grid_nlte(model, nt, ao, params=params, nthreads=16)
    assert rc == 0, f"oracle update_grid_nlte -> {rc}"
    eng = Engine(model, params=params)
    try:
        ms = eng.update_grid_nlte(nt, ag)
    finally:
        eng.close()
    return ao, ag, ms


FIELDS = ("Te", "TR", "TJ", "W", "nne", "nnetot", "nt_frac_heating", "nt_frac_ionization", "nt_frac_excitation",
          "nt_nneperion_when_solved", "totalcooling", "bin_TR", "bin_W", "bfrate_estimator", "groundlevelpop",
          "partfunct", "nlte_pops", "cooling_contrib_ion", "rates", "nt_eff_ionpot", "nt_fracdep_ionization_ion",
          "nt_prob_num_auger", "nt_ionenfrac_num_auger", "nt_ionization_ratecoeff")


def _rel(g, o, floor):
    g = np.asarray(g, dtype=np.float64)
    o = np.asarray(o, dtype=np.float64)
    both_nan = np.isnan(g) & np.isnan(o)
    d = np.abs(g - o) / np.maximum(np.maximum(np.abs(o), np.abs(g)), floor)
    d[both_nan] = 0.
    return float(np.nanmax(d, initial=0.)) if d.size else 0.


def _report(ao, ag):
    """max relative difference per output (relative to max(|x|, floor): tiny populations compare absolutely)"""
    out = {}
    for f in FIELDS:
        g, o = getattr(ag, f), getattr(ao, f)
        if f == "nlte_pops":
            mo = o < -0.9
            assert np.array_equal(mo, g < -0.9), "NLTE solution markers differ"
            g, o = g[~mo], o[~mo]
        floor = POP_ATOL if f in ("groundlevelpop", "nlte_pops") else 1e-300
        out[f] = _rel(g, o, floor)
    return out


def _compare(ao, ag, cells, tol, default):
    assert np.array_equal(ag.iters, ao.iters), (ag.iters[cells], ao.iters[cells])
    assert np.array_equal(ag.nt_timestep_last_solved, ao.nt_timestep_last_solved)
    rep = _report(ao, ag)
    print("  max rel diff: " + ", ".join(f"{k} {v:.1e}" for k, v in rep.items() if v > 0))
    bad = {k: v for k, v in rep.items() if v > tol.get(k, default)}
    assert not bad, f"outside tolerance: {bad}"


# tolerances: PINNED -- the T_e search interval holds no root, so call_T_e_finder returns the same end point on both
# sides and every output is a deterministic function of the same inputs (differences: device libm last bits through
# the LU solves); FREE -- T_e is a Brent root to TEMPERATURE_SOLVER_ACCURACY (1e-3), whose iterates a last-bit
# difference can move anywhere inside that bracket, and every T_e-dependent output follows
PINNED_TOL = {"bin_TR": 1e-3, "bin_W": 1e-2}  # find_T_R is itself a Brent root to 1e-4
PINNED_DEFAULT = 1e-6
FREE_TOL = {"Te": 1e-3, "bin_TR": 1e-3}
FREE_DEFAULT = 5e-2


def _onezone_case(first_rf, pinned):
    m = _onezone()
    nts = 6
    p = ffi.RunParams.from_buffer_copy(m.params)
    p.first_nlte_radfield_timestep = first_rf
    p.detailed_bf_usefromtimestep = first_rf + 1
    est = _estimators(m, p, nts - 1, 20000, seed=5)
    m.set_timestep(nts)
    nt = ffi.NtDataHandle(m)
    arr = ffi.NlteArrays(m, nts, est=est, dep_scale=3e-4)
    arr.params.num_lte_timesteps = 4
    if pinned:
        arr.params.T_min, arr.params.T_max = 15000., 15001.
    return m, p, nt, arr, nts


@pytest.mark.parametrize("first_rf", [12, 4])
def test_update_grid_nlte_onezone_pinned(first_rf):
    """The nebularonezone reference model at timestep 6 (NUM_LTE_TIMESTEPS 4) with a T_e interval holding no root:
    the Spencer-Fano solution, the NLTE rate matrices and their LU solves, the partition functions, electron
    densities and cooling rates of every pass agree to PINNED_DEFAULT.  first_rf = 4: the rate matrices and bf-heating
    integrals use the fitted bins (FIRST_NLTE_RADFIELD_TIMESTEP, DETAILED_BF_ESTIMATORS_USEFROMTIMESTEP)."""
    m, p, nt, arr, nts = _onezone_case(first_rf, pinned=True)
    ao, ag, ms = _solve_both(m, p, arr, nt)
    cells = arr.mgi_list
    print(f"onezone pinned first_rf={first_rf}: gpu {ms:.1f} ms, passes {ag.iters[cells]}, T_e {ag.Te[cells]}")
    assert (ao.nt_timestep_last_solved[cells] == nts).all()
    tol = dict(PINNED_TOL)
    default = PINNED_DEFAULT if first_rf > nts else 1e-3  # the bins' T_R (a Brent root) enter every rate
    _compare(ao, ag, cells, tol, default)


@pytest.mark.parametrize("first_rf", [12, 4])
def test_update_grid_nlte_onezone(first_rf):
    """The same model with the full T_e interval: the NLTE loop converges in a few passes; T_e agrees to the
    solver accuracy and the rest to FREE_DEFAULT."""
    m, p, nt, arr, nts = _onezone_case(first_rf, pinned=False)
    ao, ag, ms = _solve_both(m, p, arr, nt)
    cells = arr.mgi_list
    print(f"onezone first_rf={first_rf}: gpu {ms:.1f} ms, passes {ag.iters[cells]}, T_e {ag.Te[cells]} "
          f"(oracle {ao.Te[cells]}), f_heat {ag.nt_frac_heating[cells]}")
    assert (ao.iters[cells] > 1).all() and (ao.nt_timestep_last_solved[cells] == nts).all()
    _compare(ao, ag, cells, FREE_TOL, FREE_DEFAULT)


def test_update_grid_nlte_multicell_lte_branch():
    """A 6-shell synthetic nebular model: every non-empty cell at once, a third of them thick (the LTE branch of
    update_grid_cell, T_e = T_J and LTE ionisation) and a non-thermal skip timestep (nts < NUM_LTE_TIMESTEPS + 1:
    the Spencer-Fano defaults)."""
    m = Model(**NEB)
    nts = 5
    p = ffi.RunParams.from_buffer_copy(m.params)
    est = _estimators(m, p, nts - 1, 8000, seed=7)
    m.set_timestep(nts)
    nt = ffi.NtDataHandle(m)
    arr = ffi.NlteArrays(m, nts, est=est, seed=11, thick_frac=0.35)
    arr.params.num_lte_timesteps = 8
    ao, ag, ms = _solve_both(m, p, arr, nt)
    cells = arr.mgi_list
    print(f"multicell: gpu {ms:.1f} ms for {len(cells)} cells, passes {ag.iters[cells]}")
    assert (ao.iters[cells][arr.thick[cells] == 1] == 0).all()
    _compare(ao, ag, cells, FREE_TOL, FREE_DEFAULT)


def test_update_grid_nlte_subset_roundtrip():
    """Cells not listed come back unchanged; the listed ones match the oracle."""
    m = Model(**NEB)
    nts = 12
    p = ffi.RunParams.from_buffer_copy(m.params)
    est = _estimators(m, p, nts - 1, 8000, seed=8)
    m.set_timestep(nts)
    nt = ffi.NtDataHandle(m)
    arr = ffi.NlteArrays(m, nts, est=est, seed=12)
    arr.params.num_lte_timesteps = 2
    full = arr.mgi_list.copy()
    arr.mgi_list = full[::8].copy()
    before = arr.copy()
    ao, ag, ms = _solve_both(m, p, arr, nt)
    print(f"subset: gpu {ms:.1f} ms for {len(arr.mgi_list)} cells")
    _compare(ao, ag, arr.mgi_list, FREE_TOL, FREE_DEFAULT)
    untouched = np.setdiff1d(np.arange(m.npts_model), arr.mgi_list)
    for f in ("Te", "nne", "TR", "W"):
        assert np.array_equal(getattr(ag, f)[untouched], getattr(before, f)[untouched]), f
