"""spec.out / light_curve.out writers for the device-binned spectra (artis_gpu_spectrum).

Formats follow the reference writers exactly: write_spectrum (spectrum.cc:172-186): a header row "0 t_mid/DAY..."
then one row per frequency bin "nu_center flux(t0) flux(t1) ..."; write_light_curve (light_curve.cc:9-32):
rows "t_mid/DAY lum/LSUN lumcmf/LSUN" then the gamma-deposition / cmf_lum block.  printf("%g ") formatting.
"""
import numpy as np

DAY = 86400.0
LSUN = 3.826e33


def bin_edges(nnubins, nu_min, nu_max):
    """lower_freq and delta_freq of init_spectra (spectrum.cc:491-500)."""
    dlognu = (np.log(nu_max) - np.log(nu_min)) / nnubins
    k = np.arange(nnubins)
    lower = np.exp(np.log(nu_min) + k * dlognu)
    delta = np.exp(np.log(nu_min) + (k + 1) * dlognu) - lower
    return lower, delta


def _g(x):
    return "%g" % x


def write_spec_out(path, ts_mid, spec, nu_min, nu_max, numtimesteps=None):
    nt = spec.shape[0] if numtimesteps is None else numtimesteps
    lower, delta = bin_edges(spec.shape[1], nu_min, nu_max)
    with open(path, "w") as f:
        f.write(" ".join([_g(0.0)] + [_g(ts_mid[p] / DAY) for p in range(nt)]) + " \n")
        for nnu in range(spec.shape[1]):
            f.write(" ".join([_g(lower[nnu] + delta[nnu] / 2)] + [_g(spec[p, nnu]) for p in range(nt)]) + " \n")


def write_light_curve(path, ts_mid, ts_width, lc, lccmf, gamma_dep=None, cmf_lum=None, numtimesteps=None):
    nt = len(lc) if numtimesteps is None else numtimesteps
    gamma_dep = np.zeros(nt) if gamma_dep is None else gamma_dep
    cmf_lum = np.zeros(nt) if cmf_lum is None else cmf_lum
    with open(path, "w") as f:
        for t in range(nt):
            f.write(f"{_g(ts_mid[t] / DAY)} {_g(lc[t] / LSUN)} {_g(lccmf[t] / LSUN)}\n")
        for t in range(nt):
            f.write(f"{_g(ts_mid[t] / DAY)} {_g(gamma_dep[t] / LSUN / ts_width[t])} "
                    f"{_g(cmf_lum[t] / ts_width[t] / LSUN)}\n")
