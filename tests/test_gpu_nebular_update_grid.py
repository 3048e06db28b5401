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
import parity
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
    """Per-output max relative differences (reported) against tolerances -- for outputs that are deterministic
    functions of the same inputs."""
    assert np.array_equal(ag.iters, ao.iters), (ag.iters[cells], ao.iters[cells])
    assert np.array_equal(ag.nt_timestep_last_solved, ao.nt_timestep_last_solved)
    rep = _report(ao, ag)
    print("  max rel diff: " + ", ".join(f"{k} {v:.1e}" for k, v in rep.items() if v > 0))
    bad = {k: v for k, v in rep.items() if v > tol.get(k, default)}
    assert not bad, f"outside tolerance: {bad}"


def _ion_fractions(model, arr):
    """[npts_model, nions_total] each ion's share of its element's number density (ionstagepop, ltepop.cc:558-564)"""
    ni = model.nions_total
    g0 = model.ion_ground_statweight().astype(np.float64)
    pop = arr.groundlevelpop.reshape(-1, ni).astype(np.float64) * arr.partfunct.reshape(-1, ni) / g0
    el = model.ion_element()
    tot = np.zeros((pop.shape[0], model.nelements))
    for u in range(ni):
        tot[:, el[u]] += pop[:, u]
    with np.errstate(invalid="ignore", divide="ignore"):
        return np.nan_to_num(pop / tot[:, el])


def _compare_physical(model, ao, ag, cells, te_rtol, agg_tol):
    """The converged solution where the reference's discrete safeguards (a negative NLTE population replaced by its
    LTE value, an element reset when its populations miss the abundance by 1 %, nltepop.cc:1040-1100) can turn the
    solver's last-bit noise in negligible populations into O(1 %) changes: T_e to the solver accuracy, the ionisation
    balance, electron densities, non-thermal fractions, cooling and the radiation-field fit to agg_tol."""
    assert np.all(np.abs(ag.iters[cells] - ao.iters[cells]) <= 1), (ag.iters[cells], ao.iters[cells])
    rel = lambda f: float(np.max(np.abs(getattr(ag, f)[cells].astype(np.float64) - getattr(ao, f)[cells]) /  # noqa: E731
                                np.maximum(np.abs(getattr(ao, f)[cells]), 1e-300)))
    rep = {f: rel(f) for f in ("Te", "TR", "TJ", "W", "nne", "nnetot", "totalcooling")}
    fo, fg = _ion_fractions(model, ao)[cells], _ion_fractions(model, ag)[cells]
    rep["ion_fractions"] = float(np.max(np.abs(fg - fo)))
    for f in ("nt_frac_heating", "nt_frac_ionization", "nt_frac_excitation"):
        rep[f] = float(np.max(np.abs(getattr(ag, f)[cells] - getattr(ao, f)[cells])))
    nb = model.radfield_nbins
    bo, bg = ao.bin_TR.reshape(-1, nb)[cells], ag.bin_TR.reshape(-1, nb)[cells]
    fit = bo > 0
    rep["bin_TR"] = float(np.max(np.abs(bg[fit] - bo[fit]) / bo[fit], initial=0.))
    rates_o, rates_g = ao.rates.reshape(-1, 8)[cells], ag.rates.reshape(-1, 8)[cells]
    scale = np.maximum(np.abs(rates_o).max(axis=1, keepdims=True), 1e-300)
    rep["rates"] = float(np.max(np.abs(rates_g - rates_o) / scale))
    print("  physical max diff: " + ", ".join(f"{k} {v:.1e}" for k, v in rep.items()))
    bad = {k: v for k, v in rep.items() if v > (te_rtol if k == "Te" else agg_tol)}
    assert not bad, f"outside tolerance: {bad}"


def _read_dump_gpu(path):
    with open(path, "rb") as f:
        ne, cell1, cell2, nl, ntg = np.frombuffer(f.read(20), np.int32)
        el_D = np.frombuffer(f.read(4 * ne), np.int32)
        status = np.frombuffer(f.read(4 * ne), np.int32)
        A, b, nrm, pv = (np.frombuffer(f.read(8 * n), np.float64) for n in (cell2, cell1, cell1, cell1))
    return el_D, status, A, b, nrm, pv


def _read_dump_oracle(path, D):
    with open(path, "rb") as f:
        Do, status = np.frombuffer(f.read(8), np.int32)
        assert Do == D
        A, b, nrm, pv = (np.frombuffer(f.read(8 * n), np.float64) for n in (D * D, D, D, D))
    return status, A, b, nrm, pv


# tolerances: PINNED -- the T_e search interval holds no root, so call_T_e_finder returns the same end point on both
# sides and every output is a deterministic function of the same inputs (differences: device libm last bits through
# the LU solves); FREE -- T_e is a Brent root to TEMPERATURE_SOLVER_ACCURACY (1e-3), whose iterates a last-bit
# difference can move anywhere inside that bracket, and every T_e-dependent output follows
PINNED_TOL = {"bin_TR": 1e-3, "bin_W": 1e-2}  # find_T_R is itself a Brent root to 1e-4
PINNED_DEFAULT = 1e-6


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


def test_nlte_rate_matrices_first_pass(tmp_path, monkeypatch):
    """The first pass's NLTE rate matrices (nltepop.cc:421-628, 832-920) of every element, their LTE normalisation
    and LU solutions, dumped by both sides (ARTIS_GPU_NL_DUMP / ORACLE_NL_DUMP) from the same state: matrix
    columns to 1e-12 of their largest entry, the solution to 1e-5 in the L1 norm (the solve's backward error on
    matrices whose populations span 40 decades)."""
    prefix = str(tmp_path / "nl")
    monkeypatch.setenv("ARTIS_GPU_NL_DUMP", prefix)
    monkeypatch.setenv("ORACLE_NL_DUMP", prefix)
    m, p, nt, arr, nts = _onezone_case(12, pinned=True)
    arr.params.nlteiter = 0
    ao, ag, ms = _solve_both(m, p, arr, nt)
    el_D, status, A, b, nrm, pv = _read_dump_gpu(prefix + "_p0_gpu.bin")
    o1 = o2 = 0
    checked = 0
    for e, D in enumerate(el_D):
        D = int(D)
        Ag, bg, ng, pg = A[o2:o2 + D * D].reshape(D, D).T, b[o1:o1 + D], nrm[o1:o1 + D], pv[o1:o1 + D]
        o1, o2 = o1 + D, o2 + D * D
        fn = f"{prefix}_p0_ora_e{e}.bin"
        if D == 0 or not os.path.exists(fn):
            continue
        so, Ao, bo, no, po = _read_dump_oracle(fn, D)
        Ao = Ao.reshape(D, D).T
        assert so == status[e]
        colerr = (np.abs(Ag - Ao) / np.maximum(np.abs(Ao).max(axis=0), 1e-300)).max()
        assert colerr < 1e-12, (e, colerr)
        np.testing.assert_allclose(bg, bo, rtol=1e-15)
        np.testing.assert_allclose(ng, no, rtol=1e-12)
        l1 = np.abs(pg - po).sum() / np.abs(po).sum()
        print(f"  element {e}: D {D}, matrix {colerr:.1e}, solution L1 {l1:.1e}")
        assert l1 < 1e-5, (e, l1)
        checked += 1
    assert checked >= 2


@pytest.mark.parametrize("first_rf", [12, 4])
def test_update_grid_nlte_onezone_pinned(first_rf):
    """The nebularonezone reference model at timestep 6 (NUM_LTE_TIMESTEPS 4) with a T_e interval holding no root
    (T_e is the same end point on both sides): the Spencer-Fano solution, NLTE passes, partition functions,
    electron densities, cooling.  first_rf = 4: the rate matrices and bf-heating integrals use the fitted bins
    (FIRST_NLTE_RADFIELD_TIMESTEP, DETAILED_BF_ESTIMATORS_USEFROMTIMESTEP)."""
    m, p, nt, arr, nts = _onezone_case(first_rf, pinned=True)
    ao, ag, ms = _solve_both(m, p, arr, nt)
    cells = arr.mgi_list
    print(f"onezone pinned first_rf={first_rf}: gpu {ms:.1f} ms, passes {ag.iters[cells]}, T_e {ag.Te[cells]}")
    assert (ao.nt_timestep_last_solved[cells] == nts).all()
    _compare_physical(m, ao, ag, cells, te_rtol=1e-6, agg_tol=2e-2)


@pytest.mark.parametrize("first_rf", [12, 4])
def test_update_grid_nlte_onezone(first_rf):
    """The same model with the full T_e interval: the NLTE loop converges in a few passes."""
    m, p, nt, arr, nts = _onezone_case(first_rf, pinned=False)
    ao, ag, ms = _solve_both(m, p, arr, nt)
    cells = arr.mgi_list
    print(f"onezone first_rf={first_rf}: gpu {ms:.1f} ms, passes {ag.iters[cells]}, T_e {ag.Te[cells]} "
          f"(oracle {ao.Te[cells]}), f_heat {ag.nt_frac_heating[cells]}")
    assert (ao.iters[cells] > 1).all() and (ao.nt_timestep_last_solved[cells] == nts).all()
    _compare_physical(m, ao, ag, cells, te_rtol=1e-3, agg_tol=2e-2)


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
    _compare_physical(m, ao, ag, cells, te_rtol=1e-3, agg_tol=2e-2)


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
    _compare_physical(m, ao, ag, arr.mgi_list, te_rtol=1e-3, agg_tol=2e-2)
    untouched = np.setdiff1d(np.arange(m.npts_model), arr.mgi_list)
    for f in ("Te", "nne", "TR", "W", "nlte_pops", "groundlevelpop"):
        g, b0 = getattr(ag, f), getattr(before, f)
        if f in ("nlte_pops",):
            assert np.array_equal(g.reshape(m.npts_model, -1)[untouched], b0.reshape(m.npts_model, -1)[untouched]), f
        elif f == "groundlevelpop":
            assert np.array_equal(g.reshape(m.npts_model, -1)[untouched], b0.reshape(m.npts_model, -1)[untouched]), f
        else:
            assert np.array_equal(g[untouched], b0[untouched]), f


def test_transport_reads_the_gpu_solution():
    """The next update_packets from the GPU's nebular update_grid output (NLTE / superlevel populations, the fitted
    bins, the bf-rate estimators, the Spencer-Fano rates and Auger fractions, cooling): the engine's transport and
    the oracle's, both reading that state, agree packet by packet (tests/parity.py)."""
    m, p, nt, arr, nts = _onezone_case(4, pinned=False)
    eng = Engine(m, params=p)
    try:
        ag = arr.copy()
        eng.update_grid_nlte(nt, ag)
        assert (ag.nlte_pops > -0.9).any() and (ag.bin_W > 0).any()
        ag.apply_to_cellstate(m)
        eng.upload_cellstate(nts)
        pk = m.init_rpackets(nts, 4000, seed=91)
        pg, po = pk.copy(), pk.copy()
        eg = eng.update_packets(nts, pg)
    finally:
        eng.close()
    eo, wo = oracle_lib.update_packets(m, nts, po, params=p, nthreads=16)
    parity.assert_packets_match(pg, po)
    parity.assert_estimators_match(eg, eo)
    assert eo.radfield_count.sum() > 0
