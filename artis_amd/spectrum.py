"""Spectrum and light-curve output files for the device-binned spectra (artis_gpu_spectrum / artis_gpu_spectra).

The writers are the C++ ones of libartis_io (include/artis_io.h: artis_write_spectrum, artis_write_specpol,
artis_write_light_curve), in the formats of write_spectrum / write_specpol (spectrum.cc:144-298) and
write_light_curve (light_curve.cc:9-32).
"""
import ctypes as C

import numpy as np

from . import io as aio

DAY = 86400.0
LSUN = 3.826e33


def bin_edges(nnubins, nu_min, nu_max):
    """lower_freq and delta_freq of init_spectra (spectrum.cc:491-500): float arrays (spectrum.h:18-19)."""
    dlognu = (np.log(nu_max) - np.log(nu_min)) / nnubins
    k = np.arange(nnubins)
    lower = np.exp(np.log(nu_min) + k * dlognu).astype(np.float32)
    delta = (np.exp(np.log(nu_min) + (k + 1) * dlognu) - lower.astype(np.float64)).astype(np.float32)
    return lower.astype(np.float64), delta.astype(np.float64)


def _dp(a):
    return None if a is None else a.ctypes.data_as(C.POINTER(C.c_double))


def _lib():
    L = aio.lib()
    dp = C.POINTER(C.c_double)
    L.artis_write_spectrum.argtypes = [C.c_char_p] * 4 + [C.c_int, C.c_int, dp, C.c_int, C.c_double, C.c_double,
                                                          C.c_int, C.c_int, dp, dp, dp, dp]
    L.artis_write_specpol.argtypes = [C.c_char_p] * 3 + [C.c_int, dp, C.c_int, C.c_double, C.c_double, C.c_int,
                                                         C.c_int, dp, dp, dp]
    L.artis_write_light_curve.argtypes = [C.c_char_p, C.c_int, C.c_int, dp, dp, dp, dp, dp, dp]
    return L


def _b(path):
    return None if path is None else str(path).encode()


def _c(x):
    return None if x is None else np.ascontiguousarray(x, dtype=np.float64)


def write_spec_out(path, ts_mid, spec, nu_min, nu_max, numtimesteps=None, emission=None, trueemission=None,
                   absorption=None, emission_path=None, trueemission_path=None, absorption_path=None):
    """spec.out (and emission.out / emissiontrue.out / absorption.out when their arrays and paths are given)."""
    keep = [_c(x) for x in (ts_mid, spec, emission, trueemission, absorption)]
    nt, nnb = keep[1].shape
    n = nt if numtimesteps is None else numtimesteps
    proccount = emission.shape[-1] if emission is not None else 0
    ioncount = absorption.shape[-1] if absorption is not None else 0
    rc = _lib().artis_write_spectrum(_b(path), _b(emission_path), _b(trueemission_path), _b(absorption_path), nt, n,
                                     _dp(keep[0]), nnb, nu_min, nu_max, proccount, ioncount, _dp(keep[1]),
                                     _dp(keep[2]), _dp(keep[3]), _dp(keep[4]))
    if rc != 0:
        raise OSError(f"artis_write_spectrum({path}) -> {rc}")


def write_specpol(path, ts_mid, stokes_flux, nu_min, nu_max, stokes_emission=None, stokes_absorption=None,
                  emission_path=None, absorption_path=None):
    """specpol.out (and emissionpol.out / absorptionpol.out)."""
    keep = [_c(x) for x in (ts_mid, stokes_flux, stokes_emission, stokes_absorption)]
    _, nt, nnb = keep[1].shape
    proccount = stokes_emission.shape[-1] if stokes_emission is not None else 0
    ioncount = stokes_absorption.shape[-1] if stokes_absorption is not None else 0
    rc = _lib().artis_write_specpol(_b(path), _b(emission_path), _b(absorption_path), nt, _dp(keep[0]), nnb, nu_min,
                                    nu_max, proccount, ioncount, _dp(keep[1]), _dp(keep[2]), _dp(keep[3]))
    if rc != 0:
        raise OSError(f"artis_write_specpol({path}) -> {rc}")


def write_light_curve(path, ts_mid, ts_width, lc, lccmf, gamma_dep=None, cmf_lum=None, numtimesteps=None, abin=-1):
    nt = len(lc) if numtimesteps is None else numtimesteps
    keep = [_c(x) for x in (ts_mid, ts_width, lc, lccmf, gamma_dep, cmf_lum)]
    rc = _lib().artis_write_light_curve(_b(path), abin, nt, *[_dp(k) for k in keep])
    if rc != 0:
        raise OSError(f"artis_write_light_curve({path}) -> {rc}")
