// spectrum.h -- emergent spectrum and light curve of the escaped r-packets, binned on the device.
//
// The binning of write_partial_lightcurve_spectra (spectrum.cc:641-721): every packet with type TYPE_ESCAPE and
// escape_type TYPE_RPKT goes through add_to_lc_res (light_curve.cc:34-54) and add_to_spec (spectrum.cc:339-362),
// angle-averaged (abin -1), without the emission-resolved columns.  Sums are float64 atomics; the reference's
// serial loop adds in packet order, so sums agree to rounding (tests/test_spectrum.py).
#ifndef ARTIS_SPECTRUM_H
#define ARTIS_SPECTRUM_H

#include "physics.h"

// sn3d.h:168-180 get_timestep (linear search, as the reference)
DEVFN int spec_timestep(const Ctx &K, int ntstep, double t) {
  for (int nts = 0; nts < ntstep; nts++) {
    const double tsend = (nts < ntstep - 1) ? K.G.ts_start[nts + 1] : K.G.tmax;
    if (t >= K.G.ts_start[nts] && t < tsend) return nts;
  }
  return -1;
}

__global__ void k_spectrum(const Ctx *__restrict__ ctxp, const uint64_t *__restrict__ soa, int64_t n, int ntstep,
                           int nnubins, double dlognu, const double *__restrict__ delta_freq, double nprocs,
                           double *spec, double *lc_lum, double *lc_lumcmf) {
  const Ctx &K = *ctxp;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (hi32(soa[PW(n, i, 0)]) != ARTIS_TYPE_ESCAPE) return;
  const uint64_t w32 = soa[PW(n, i, 32)];
  if (lo32(w32) != ARTIS_TYPE_RPKT) return;
  const int escape_time = hi32(w32);
  const double pos[3] = {asd(soa[PW(n, i, 3)]), asd(soa[PW(n, i, 4)]), asd(soa[PW(n, i, 5)])};
  const double dir[3] = {asd(soa[PW(n, i, 6)]), asd(soa[PW(n, i, 7)]), asd(soa[PW(n, i, 8)])};
  const double e_cmf = asd(soa[PW(n, i, 9)]);
  const double e_rf = asd(soa[PW(n, i, 10)]);
  const double nu_rf = asd(soa[PW(n, i, 12)]);
  const double tmin = K.G.tmin, tmax = K.G.tmax;
  // light_curve.cc:39-52 (vectors.h:146-156 get_arrive_time / get_arrive_time_cmf)
  const double t_arrive = escape_time - (dot(pos, dir) / ARTIS_CLIGHT_PROP);
  if (t_arrive > tmin && t_arrive < tmax) {
    const int nt = spec_timestep(K, ntstep, t_arrive);
    if (nt >= 0) unsafeAtomicAdd(&lc_lum[nt], e_rf / K.G.ts_width[nt] / nprocs);
  }
  const double cmfcorr = sqrt(1. - (K.G.vmax * K.G.vmax / ARTIS_CLIGHTSQUARED));
  const double t_arrive_cmf = escape_time * cmfcorr;
  if (t_arrive_cmf > tmin && t_arrive_cmf < tmax) {
    const int nt = spec_timestep(K, ntstep, t_arrive_cmf);
    if (nt >= 0) unsafeAtomicAdd(&lc_lumcmf[nt], e_cmf / K.G.ts_width[nt] / nprocs / cmfcorr);
  }
  // spectrum.cc:348-362
  const double nu_min = K.G.nu_min_r, nu_max = K.G.nu_max_r;
  if (t_arrive > tmin && t_arrive < tmax && nu_rf > nu_min && nu_rf < nu_max) {
    const int nt = spec_timestep(K, ntstep, t_arrive);
    const int nnu = (int)((log(nu_rf) - log(nu_min)) / dlognu);
    if (nt >= 0 && nnu >= 0 && nnu < nnubins) {
      const double deltaE =
          e_rf / K.G.ts_width[nt] / delta_freq[nnu] / 4.e12 / ARTIS_PI / ARTIS_PARSEC / ARTIS_PARSEC / nprocs;
      unsafeAtomicAdd(&spec[(int64_t)nt * nnubins + nnu], deltaE);
    }
  }
}

#endif
