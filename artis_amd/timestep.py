"""The body of sn3d.cc's do_timestep (sn3d.cc:514-673) for the LTE-population options with every per-timestep
stage on the device: update_grid's estimator preparation and temperature / ionisation solution
(artis_gpu_prepare_temperatures + artis_gpu_solve_temperatures, update_grid.cc:1041-1205), the per-cell tables
(artis_gpu_upload_cellstate, the cellhistory replacement) and the packet propagation
(artis_gpu_update_packets_resident, sn3d.cc:574) with the packets resident in HBM across timesteps.

Host work per timestep is what the reference's host does between those calls: the raw estimators come back
(D2H, a few MB), the solved cell state goes into the model's cell-state arrays, and the per-cell tables are
uploaded.  Cell quantities the LTE update_grid does not solve for -- the density at the new time, the grey opacity
and thick-cell flag (update_grid.cc:1012-1040, 1162-1212: host bookkeeping) -- come from the synthetic model's
artis_model_advance (model_synth.cc: rho(t) and the grey-depth rule, without recomputing the rest of its synthetic
cell state); the abundances of the synthetic models do not decay.
"""
import ctypes as C
import time

import numpy as np

from . import ffi


def _f32(p, n):
    return np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_float)), (n,))


def _f64(p, n):
    return np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_double)), (n,))


def _copy_arrays(obj):
    import copy

    o = copy.copy(obj)
    for k, v in obj.__dict__.items():
        if isinstance(v, np.ndarray):
            setattr(o, k, v.copy())
    return o


class LteTimestepLoop:
    """update_grid (GPU) -> upload_cellstate -> update_packets (resident) over consecutive timesteps."""

    def __init__(self, model, eng, rank=0, keep_inputs=False):
        """keep_inputs: keep a copy of each update_grid's inputs (last_inputs, for an oracle replay in the tests)."""
        self.m, self.eng, self.rank = model, eng, rank
        self.keep_inputs = keep_inputs
        self.last_inputs = None
        g = ffi.Geometry.from_address(model.geometry)
        self.vol_init = ffi.model_vol_init(model).astype(np.float64)  # vol_init_modelcell (grid.cc:94-110)
        self.ts_mid = np.ctypeslib.as_array(g.ts_mid, (g.ntstep,)).copy()
        self.ts_width = np.ctypeslib.as_array(g.ts_width, (g.ntstep,)).copy()
        self.tmin = g.tmin
        self.solution = None

    def radiation_energy(self, nts):
        """Sum over model cells of a W T_R^4 V(t): the radiation energy the cell state's dilute black body holds at
        the start of timestep nts.  Packets initialised with this total energy give estimators whose normalised J
        matches the cell state, so update_grid's thermal balance has roots inside [MINTEMP, MAXTEMP]."""
        a_rad = 7.5657e-15
        cs = self._cell_arrays()
        g = ffi.Geometry.from_address(self.m.geometry)
        t = np.ctypeslib.as_array(g.ts_start, (g.ntstep,))[nts]
        vol = self.vol_init * (t / self.tmin) ** 3
        return float(np.sum(a_rad * cs["W"].astype(np.float64) * cs["TR"].astype(np.float64) ** 4 * vol))

    def _cell_arrays(self):
        m = self.m
        cs = ffi.CellState.from_address(m.cellstate)
        np_, nel, ni, mx = m.npts_model, m.nelements, m.nions_total, m.maxnions
        return {"Te": _f32(cs.Te, np_), "TR": _f32(cs.TR, np_), "TJ": _f32(cs.TJ, np_), "W": _f32(cs.W, np_),
                "nne": _f32(cs.nne, np_), "nnetot": _f32(cs.nnetot, np_),
                "groundlevelpop": _f32(cs.groundlevelpop, np_ * ni), "partfunct": _f32(cs.partfunct, np_ * ni),
                "totalcooling": _f64(cs.totalcooling, np_), "cooling_contrib_ion": _f64(cs.cooling_contrib_ion, np_ * ni),
                "corrphotoionrenorm": _f64(cs.corrphotoionrenorm, np_ * nel * mx)}

    def update_grid(self, nts, est):
        """update_grid for timestep nts from the raw estimators `est` of timestep nts - 1 (update_grid.cc:1316 pairs
        them): the density / opacity for nts (artis_model_advance), then the GPU preparation and solution on every
        non-empty cell; the solved state is written into the model's cell-state arrays.  Returns device milliseconds."""
        m, eng = self.m, self.eng
        tp = {}
        t = time.perf_counter()
        prev = {k: v.copy() for k, v in self._cell_arrays().items()}
        m.advance(nts)  # rho(t), kappagrey, thick at nts (host bookkeeping)
        tp["advance"] = (time.perf_counter() - t) * 1e3
        # nts_for_te = nts - 1 (update_grid.cc:804)
        te = ffi.TeArrays(m, t_current=float(self.ts_mid[nts - 1]), synthetic=False)
        # the previous timestep's solution is the solver's starting state (the reference's modelgrid values)
        for k in ("TR", "W", "TJ", "Te"):
            setattr(te, k, prev[k].copy())
        te.groundlevelpop = prev["groundlevelpop"].copy()
        te.vol_init = self.vol_init.copy()
        te.thick = np.ctypeslib.as_array(C.cast(ffi.CellState.from_address(m.cellstate).thick, C.POINTER(C.c_int16)),
                                         (m.npts_model,)).copy()
        te.mgi_list = np.nonzero((te.rho > 0) & (self.vol_init > 0))[0].astype(np.int32)
        if self.solution is not None:
            # cells in the order of their previous solution's Brent iteration count: a wave of k_te_solve runs as
            # many thermal-balance evaluations as its slowest cell needs, and a cell's count changes little from one
            # timestep to the next (the order changes no result: the cells are independent)
            prev_iters = self.solution.iters[te.mgi_list]
            te.mgi_list = te.mgi_list[np.argsort(prev_iters, kind="stable")]
        ug = ffi.UgArrays(m, deltat=float(self.ts_width[nts - 1]), tratmid=float(self.ts_mid[nts] / self.tmin),
                          synthetic=False)
        ug.J, ug.nuJ, ug.ffheating, ug.colheating = est.J, est.nuJ, est.ffheating, est.colheating
        ug.gamma, ug.bfheating = est.gamma, est.bfheating
        ug.nne, ug.partfunct = prev["nne"].copy(), prev["partfunct"].copy()
        if self.keep_inputs:
            self.last_inputs = (te.copy(), _copy_arrays(ug))  # for an oracle replay (tests)
        t1 = time.perf_counter()
        tp["inputs"] = (t1 - t) * 1e3 - tp["advance"]
        t = t1
        eng.prepare_temperatures(te, ug)
        tp["prepare"] = (time.perf_counter() - t) * 1e3
        te.TR, te.W, te.TJ = ug.TR_out, ug.W_out, ug.TJ_out
        te.ffheating, te.colheating, te.gamma, te.bfheating = ug.ff_out, ug.col_out, ug.gamma_out, ug.bfheating_out
        t2 = time.perf_counter()
        ms = eng.solve_temperatures(te)
        tp["solve"] = (time.perf_counter() - t2) * 1e3
        host_ms = (time.perf_counter() - t) * 1e3
        cur = self._cell_arrays()
        g = te.mgi_list
        for k in ("Te", "TR", "TJ", "W", "nne", "nnetot", "totalcooling"):
            cur[k][g] = getattr(te, k)[g]
        ni, nel, mx = m.nions_total, m.nelements, m.maxnions
        rows = (g[:, None] * ni + np.arange(ni)[None, :]).ravel()
        cur["groundlevelpop"][rows] = te.groundlevelpop[rows]
        cur["partfunct"][rows] = te.partfunct[rows]
        cur["cooling_contrib_ion"][rows] = te.cooling_contrib_ion[rows]
        rr = (g[:, None] * nel * mx + np.arange(nel * mx)[None, :]).ravel()
        cur["corrphotoionrenorm"][rr] = ug.renorm_out[rr]
        tp["writeback"] = (time.perf_counter() - t) * 1e3 - host_ms
        self.last_parts_ms = tp
        self.solution = te
        return ms, host_ms

    def run(self, nts0, nsteps, progress=None):
        """Timesteps nts0 .. nts0 + nsteps - 1 of the resident packets (uploaded by the caller).  The first one
        propagates on the cell state the model holds; every later one first runs update_grid from the previous
        step's estimators.  Returns one record per timestep (wall ms of the whole timestep and its parts)."""
        m, eng = self.m, self.eng
        out = []
        est = None
        for k in range(nsteps):
            nts = nts0 + k
            t0 = time.perf_counter()
            ug_ms = ug_host_ms = 0.
            if k > 0:
                ug_ms, ug_host_ms = self.update_grid(nts, est)
            t1 = time.perf_counter()
            eng.upload_cellstate(nts)
            eng.zero_estimators()
            eng.step_resident(nts, my_rank=self.rank)
            est = eng.download_estimators()
            t2 = time.perf_counter()
            rec = {"nts": nts, "ms": (t2 - t0) * 1e3, "update_grid_ms": (t1 - t0) * 1e3, "update_grid_gpu_ms": ug_ms,
                   "precompute_ms": eng.last_precompute_ms(), "transport_ms": eng.last_transport_ms(),
                   "nesc": int(est.struct.nesc)}
            if k > 0:
                te = self.solution
                rec["update_grid_parts_ms"] = self.last_parts_ms
                rec["cells_solved"] = int(len(te.mgi_list))
                rec["Te_mean"] = float(np.mean(te.Te[te.mgi_list]))
            out.append(rec)
            if progress:
                progress(f"timestep loop nts {nts}: {rec['ms']:.0f} ms (update_grid {rec['update_grid_ms']:.0f})")
        return out
