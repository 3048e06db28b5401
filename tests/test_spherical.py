"""GRID_SPHERICAL1D (boundary.cc:14-99 get_shellcrossdist, the spherical branch of boundary_cross boundary.cc:101-330,
spherical1d_grid_setup grid.cc:2104-2131, the spherical maxsdist of rpkt.cc:659-661 / gammapkt.cc:551-553): the host
grid record and the oracle's propagation, checked by geometry alone.  The GPU parity tests are in
tests/test_gpu_spherical.py.

The reference has no spherical fixture of its own (every artisoptions_*.h sets GRID_UNIFORM), so the checks are the
properties a radial-shell propagation must have: a packet that ends the timestep sits inside the expanding shell its
`where` names, an escaped packet left through the outer boundary r = rmax t / tmin, and the bookkeeping invariants of
the cuboid runs (tests/test_oracle.py) hold.

One exception is the reference's own: get_shellcrossdist drops an intersection at which the ray's radial direction
has the "wrong" sign (boundary.cc:64-79) without allowing for the shell's expansion, so a ray that grazes an
expanding inner shell enters it while moving slightly outward (pos . dir > 0 at the entry point), that entry is
dropped, and the packet continues inside the inner sphere labelled with its old shell (later steps see no inner
crossing from inside).  The restatement keeps this; such packets are rare (a few per 1e4 steps) and always BELOW
their shell's inner radius, which is what the tests allow.
"""
import numpy as np
import pytest

import oracle_lib
from artis_amd import ffi
from artis_amd.model import Model

SPH = dict(nshells_1d=40, grid_spherical=1, nlevels_per_ion=40, n_ionising=15, max_lines=4000, ntstep=30)


@pytest.fixture(scope="module")
def sph_model():
    return Model(**SPH)


def _geom(m):
    g = ffi.Geometry.from_address(m.geometry)
    n = g.ngrid
    r_in = np.ctypeslib.as_array(g.cell_pos_min, (3 * n,))[0::3].copy()
    wid = np.ctypeslib.as_array(g.modelcell_wid_init, (n,)).copy()
    mgi = np.ctypeslib.as_array(g.cell_mgi, (n,)).copy()
    return g, r_in, wid, mgi


def test_spherical_grid_record(sph_model):
    g, r_in, wid, mgi = _geom(sph_model)
    assert g.grid_type == ffi.GRID_SPHERICAL1D
    assert list(g.ncoordgrid) == [40, 1, 1] and g.ngrid == sph_model.npts_model == 40
    assert r_in[0] == 0 and np.all(wid > 0)
    # shells tile [0, rmax] at tmin: each inner radius is the previous shell's outer one
    assert np.allclose(r_in[1:], (r_in + wid)[:-1], rtol=1e-14, atol=0)
    assert np.isclose(r_in[-1] + wid[-1], g.rmax, rtol=1e-14)
    assert np.array_equal(mgi, np.arange(40))
    # vol_init_modelcell of a shell (grid.cc:94-110)
    vol = ffi.model_vol_init(sph_model)
    assert np.allclose(vol, 4 / 3 * np.pi * ((r_in + wid) ** 3 - r_in ** 3), rtol=1e-14)


def _inside_shells(m, pk):
    g, r_in, wid, _ = _geom(m)
    alive = pk["type"] != ffi.TYPE_ESCAPE
    t = pk["prop_time"][alive]
    r = np.linalg.norm(pk["pos"][alive], axis=1)
    w = pk["where"][alive]
    lo = r_in[w] * t / g.tmin - 10.0  # boundary_cross's 10 cm tolerance
    hi = (r_in[w] + wid[w]) * t / g.tmin + 10.0
    return alive, r, lo, hi


def _check_shells(r, lo, hi, max_frac=0.005):
    """Every packet inside its shell except the grazing-entry packets of the module docstring: never above the outer
    radius, below the inner one for at most max_frac of them."""
    assert np.all(r <= hi), np.nonzero(r > hi)
    below = r < lo
    assert below.mean() <= max_frac, (below.sum(), len(r))
    return int(below.sum())


@pytest.mark.parametrize("nts", [4, 12])
def test_spherical_rpackets(sph_model, nts):
    m = sph_model
    m.set_timestep(nts)
    pk0 = m.init_rpackets(nts, 2500, seed=31 + nts)
    _, r, lo, hi = _inside_shells(m, pk0)
    assert np.all((r >= lo) & (r <= hi))  # the initial placement: exact
    pk = pk0.copy()
    est, work = oracle_lib.update_packets(m, nts, pk, nthreads=8)
    alive, r, lo, hi = _inside_shells(m, pk)
    _check_shells(r, lo, hi)
    g = ffi.Geometry.from_address(m.geometry)
    t2 = pk["prop_time"][alive]
    assert np.allclose(t2, t2.max(), rtol=0, atol=0)
    esc = ~alive
    assert esc.sum() > 100 and est.struct.nesc == esc.sum()
    # escaped through the outer shell's boundary, expanding with the flow
    r_esc = np.linalg.norm(pk["pos"][esc], axis=1)
    assert np.allclose(r_esc, g.rmax * pk["prop_time"][esc] / g.tmin, rtol=1e-9)
    assert np.isclose(est.struct.cmf_lum, pk["e_cmf"][esc].sum(), rtol=1e-12)
    c = est.counters
    assert c[0] + c[1] + c[4] + c[5] == c[7] + c[8] + c[9] + c[10]
    assert c[28] > 10 * len(pk)  # cell crossings (COUNTER_CELLCROSSINGS)
    assert est.J.sum() > 0


def test_spherical_pellets_and_gamma(sph_model):
    """Pellets placed in shells (place_pellet's spherical branch, packet.cc:29-38), decays, gamma rays through the
    shells (gammapkt.cc:551-553), over three timesteps."""
    m = sph_model
    pe = m.init_pellets(3000, seed=5)
    for nts in (0, 1, 2):
        m.set_timestep(nts)
        oracle_lib.update_packets(m, nts, pe, nthreads=8)
        alive, r, lo, hi = _inside_shells(m, pe)
        _check_shells(r, lo, hi)
    assert (pe["type"] == ffi.TYPE_ESCAPE).sum() > 100


def test_spherical_reference_1d_inputs():
    """The classic 1D inputs (tests/classicmode_inputfiles model.txt, 78 shells) on the spherical grid."""
    import os

    d = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ref_inputs", "classicmode")
    m = Model(files=(os.path.join(d, "input-newrun.txt"), os.path.join(d, "model.txt"), os.path.join(d, "abundances.txt")),
              grid_spherical=1, nlevels_per_ion=40, n_ionising=15, max_lines=4000)
    g, r_in, wid, mgi = _geom(m)
    assert g.grid_type == ffi.GRID_SPHERICAL1D and g.ngrid == m.npts_model
    m.set_timestep(12)
    pk = m.init_rpackets(12, 1500, seed=8)
    oracle_lib.update_packets(m, 12, pk, nthreads=8)
    alive, r, lo, hi = _inside_shells(m, pk)
    _check_shells(r, lo, hi)
