"""Emergent spectrum / light curve binning: device binning (artis_gpu_spectrum) vs the
oracle's restatement of write_partial_lightcurve_spectra, and the spec.out / light_curve.out writers."""
import numpy as np
import pytest

import oracle_lib
from artis_amd import ffi
from artis_amd.spectrum import bin_edges, write_light_curve, write_spec_out


def _escaped_packets(model, nts, n, seed):
    model.set_timestep(nts)
    pk = model.init_rpackets(nts, n, seed=seed)
    oracle_lib.update_packets(model, nts, pk)
    return pk


def test_oracle_spectrum_conserves_escaped_energy(small_model):
    """Every escaped r-packet lands in exactly one bin: sum(flux * dnu * width) * 4e12 pi pc^2 == sum e_rf."""
    pk = _escaped_packets(small_model, 9, 3000, 21)
    spec, lc, lccmf = oracle_lib.spectrum(small_model, pk)
    esc = (pk["type"] == ffi.TYPE_ESCAPE) & (pk["escape_type"] == ffi.TYPE_RPKT)
    assert esc.sum() > 50
    geom_w = _ts_width(small_model)
    lower, delta = bin_edges(1000, 1e14, 5e15)
    pc = 3.0857e18
    e_spec = (spec * delta[None, :] * geom_w[:, None]).sum() * 4.e12 * 3.1415926535987 * pc * pc
    e_lc = (lc * geom_w).sum()
    inband = esc & (pk["nu_rf"] > 1e14) & (pk["nu_rf"] < 5e15)
    assert np.isclose(e_spec, pk["e_rf"][inband].sum(), rtol=1e-10)
    assert np.isclose(e_lc, pk["e_rf"][esc].sum(), rtol=1e-10)
    assert lccmf.sum() > 0


def _ts_width(model):
    import ctypes as C

    # artis_geometry: ... tmin, tmax, rmax, vmax, ntstep, ts_start, ts_width (include/artis_gpu.h)
    class G(C.Structure):
        _fields_ = [("grid_type", C.c_int32), ("ncoordgrid", C.c_int32 * 3), ("ngrid", C.c_int32),
                    ("npts_model", C.c_int32), ("cell_pos_min", C.c_void_p), ("cell_mgi", C.c_void_p),
                    ("wid", C.c_void_p), ("coordmax", C.c_double * 3), ("tmin", C.c_double), ("tmax", C.c_double),
                    ("rmax", C.c_double), ("vmax", C.c_double), ("ntstep", C.c_int32),
                    ("ts_start", C.POINTER(C.c_double)), ("ts_width", C.POINTER(C.c_double)),
                    ("ts_mid", C.POINTER(C.c_double))]
    g = G.from_address(model.geometry)
    return np.ctypeslib.as_array(g.ts_width, shape=(g.ntstep,)).copy()


def test_writers_follow_reference_format(tmp_path, small_model):
    pk = _escaped_packets(small_model, 9, 1000, 22)
    spec, lc, lccmf = oracle_lib.spectrum(small_model, pk, nnubins=50)
    nt = spec.shape[0]
    ts_mid = np.linspace(1, 2, nt) * 86400.0
    write_spec_out(tmp_path / "spec.out", ts_mid, spec, 1e14, 5e15, numtimesteps=10)
    rows = (tmp_path / "spec.out").read_text().splitlines()
    assert len(rows) == 51 and len(rows[0].split()) == 11 and rows[0].split()[0] == "0"
    back = np.array([[float(v) for v in r.split()] for r in rows[1:]])
    assert np.allclose(back[:, 1:], spec[:10].T, rtol=1e-5)
    write_light_curve(tmp_path / "light_curve.out", ts_mid, np.ones(nt), lc, lccmf, numtimesteps=10)
    assert len((tmp_path / "light_curve.out").read_text().splitlines()) == 20


@pytest.mark.gpu
def test_device_spectrum_matches_oracle(small_model):
    from artis_amd import Engine

    nts = 9
    small_model.set_timestep(nts)
    pk = small_model.init_rpackets(nts, 4000, seed=23)
    eng = Engine(small_model)
    try:
        eng.upload_cellstate(nts)
        eng.update_packets(nts, pk)       # engine-propagated packets, now resident on the device
        spec, lc, lccmf = eng.spectrum()
    finally:
        eng.close()
    so, lo, lco = oracle_lib.spectrum(small_model, pk)  # same packets binned on the CPU
    scale = np.abs(so).sum()
    assert scale > 0
    assert np.abs(spec - so).sum() / scale < 1e-12
    assert np.allclose(lc, lo, rtol=1e-12, atol=0)
    assert np.allclose(lccmf, lco, rtol=1e-12, atol=0)


def test_oracle_spectra_resolved_columns_sum_to_flux(small_model):
    """add_to_spec_res (spectrum.cc:339-452): every escaped packet adds deltaE once to the flux and once to an
    emission / true-emission column, so the columns sum to the flux; unpolarised packets (Stokes I = 1) give
    stokes_I == flux; the 100 direction bins (weight MABINS) average to the angle-averaged spectrum."""
    pk = _escaped_packets(small_model, 9, 3000, 24)
    s = oracle_lib.spectra(small_model, pk, nnubins=200, emission_res=True, stokes=True)
    flux = s.flux
    assert flux.sum() > 0
    assert np.allclose(s.emission.sum(-1), flux, rtol=1e-12, atol=1e-300)
    assert np.allclose(s.trueemission.sum(-1), flux, rtol=1e-12, atol=1e-300)
    assert s.absorption.sum() > 0
    esc = pk["type"] == ffi.TYPE_ESCAPE
    if np.all(pk["stokes"][esc][:, 0] == 1.0):
        assert np.allclose(s.stokes_flux[0], flux, rtol=1e-12, atol=1e-300)
    assert np.allclose(s.stokes_emission[0].sum(-1), s.stokes_flux[0], rtol=1e-12, atol=1e-300)
    simple, lc, lccmf = oracle_lib.spectrum(small_model, pk, nnubins=200)
    assert np.array_equal(simple, flux) and np.array_equal(lc, s.lc_lum) and np.array_equal(lccmf, s.lc_lumcmf)
    tot = np.zeros_like(flux)
    lct = np.zeros_like(lc)
    for abin in range(ffi.MABINS):
        sa = oracle_lib.spectra(small_model, pk, nnubins=200, abin=abin, syn_dir=(0., 0., 1.), emission_res=False)
        tot += sa.flux
        lct += sa.lc_lum
        assert not sa.lc_lumcmf.any()
    assert np.allclose(tot / ffi.MABINS, flux, rtol=1e-10, atol=1e-300)
    assert np.allclose(lct / ffi.MABINS, lc, rtol=1e-10, atol=1e-300)


def test_resolved_writers_follow_reference_format(tmp_path, small_model):
    """emission.out / emissiontrue.out / absorption.out: one row per (frequency bin, timestep) of proccount /
    ioncount columns (spectrum.cc:176-200); specpol.out: header with the timesteps three times, rows
    "nu I.. Q.. U.." (spectrum.cc:232-298)."""
    from artis_amd.spectrum import write_specpol

    pk = _escaped_packets(small_model, 9, 1000, 25)
    s = oracle_lib.spectra(small_model, pk, nnubins=40, emission_res=True, stokes=True)
    nt = s.flux.shape[0]
    ts_mid = np.linspace(1, 2, nt) * 86400.0
    write_spec_out(tmp_path / "spec.out", ts_mid, s.flux, 1e14, 5e15, numtimesteps=12, emission=s.emission,
                   trueemission=s.trueemission, absorption=s.absorption, emission_path=tmp_path / "emission.out",
                   trueemission_path=tmp_path / "emissiontrue.out", absorption_path=tmp_path / "absorption.out")
    em = (tmp_path / "emission.out").read_text().splitlines()
    ab = (tmp_path / "absorption.out").read_text().splitlines()
    assert len(em) == 40 * 12 and len(em[0].split()) == s.proccount and len(ab[0].split()) == s.ioncount
    back = np.array([[float(v) for v in r.split()] for r in em]).reshape(40, 12, s.proccount)
    assert np.allclose(back, s.emission[:12].transpose(1, 0, 2), rtol=1e-5)
    write_specpol(tmp_path / "specpol.out", ts_mid, s.stokes_flux, 1e14, 5e15, s.stokes_emission,
                  s.stokes_absorption, tmp_path / "emissionpol.out", tmp_path / "absorptionpol.out")
    rows = (tmp_path / "specpol.out").read_text().splitlines()
    assert len(rows) == 41 and len(rows[0].split()) == 1 + 3 * nt
    back = np.array([[float(v) for v in r.split()] for r in rows[1:]])
    assert np.allclose(back[:, 1:1 + nt], s.stokes_flux[0].T, rtol=1e-5)
    assert np.allclose(back[:, 1 + 2 * nt:], s.stokes_flux[2].T, rtol=1e-5, atol=1e-300)
    lower, delta = bin_edges(40, 1e14, 5e15)
    assert np.allclose(back[:, 0], (lower + delta / 2), rtol=1e-5)  # "%g": 6 significant digits
    assert len((tmp_path / "emissionpol.out").read_text().splitlines()) == 40 * 3 * nt


@pytest.mark.gpu
@pytest.mark.parametrize("abin", [-1, 37])
def test_device_spectra_match_oracle(small_model, abin):
    """artis_gpu_spectra vs oracle_spectra: flux, emission / true-emission / absorption, Stokes I/Q/U and the
    light curves of the engine-propagated packets (float64 atomics vs serial sums: ESTIMATOR_RTOL)."""
    from artis_amd import Engine

    nts = 9
    small_model.set_timestep(nts)
    pk = small_model.init_rpackets(nts, 4000, seed=26)
    eng = Engine(small_model)
    try:
        eng.upload_cellstate(nts)
        eng.update_packets(nts, pk)
        g = eng.spectra(nnubins=300, abin=abin, syn_dir=(0.3, 0.4, np.sqrt(0.75)), emission_res=True, stokes=True)
    finally:
        eng.close()
    o = oracle_lib.spectra(small_model, pk, nnubins=300, abin=abin, syn_dir=(0.3, 0.4, np.sqrt(0.75)),
                           emission_res=True, stokes=True)
    for name, a in o.arrays().items():
        b = getattr(g, name)
        scale = max(np.abs(a).max(), 1e-300)
        assert np.abs(a - b).max() <= 1e-9 * scale, name
    assert o.flux.sum() > 0 and o.emission.sum() > 0
