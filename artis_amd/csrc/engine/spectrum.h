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

// ---- exspec spectra (spectrum.cc:306-452, light_curve.cc:34-62) -------------------------------------------------
struct SpecArgs {
  int nnubins, nprocs, abin, ntstep, proccount, ioncount, maxnions, nbf;
  double syn_dir[3];
  double dlognu;
  const double *delta_freq;  // [nnubins] (init_spectra, host libm)
  const int32_t *bf_col;     // [nbf] bflist index -> element * maxnions + ion (columnindex_from_emissiontype)
  const int32_t *line_elem, *line_ion;
  double *flux, *emission, *trueemission, *absorption;
  double *sflux, *semission, *sabsorption;  // Stokes I, Q, U blocks one after the other
  double *lc, *lccmf, *glc, *glccmf;
};

// spectrum.cc:306-337 columnindex_from_emissiontype
DEVFN int spec_column(const SpecArgs &A, int et) {
  if (et >= 0) return A.line_elem[et] * A.maxnions + A.line_ion[et];
  if (et == -9999999 || A.nbf == 0) return 2 * A.ioncount;
  return A.ioncount + A.bf_col[-1 - et];
}

// vectors.h:158-193 get_escapedirectionbin (NPHIBINS = NCOSTHETABINS = 10, exspec.h:7-9)
DEVFN int escapedirectionbin(const double dir_in[3], const double syn_dir[3]) {
  const double xhat[3] = {1.0, 0.0, 0.0};
  const double dirmag = sqrt((dir_in[0] * dir_in[0]) + (dir_in[1] * dir_in[1]) + (dir_in[2] * dir_in[2]));
  const double dir[3] = {dir_in[0] / dirmag, dir_in[1] / dirmag, dir_in[2] / dirmag};
  const double costheta = dot(dir, syn_dir);
  const int costhetabin = (int)((costheta + 1.0) * 10 / 2.0);
  double vec1[3], vec2[3], vec3[3];
  cross_prod(dir, syn_dir, vec1);
  cross_prod(xhat, syn_dir, vec2);
  const double cosphi = dot(vec1, vec2) / vec_len(vec1) / vec_len(vec2);
  cross_prod(vec2, syn_dir, vec3);
  const double testphi = dot(vec1, vec3);
  int phibin;
  if (testphi > 0)
    phibin = (int)(acos(cosphi) / 2. / ARTIS_PI * 10);
  else
    phibin = (int)((acos(cosphi) + ARTIS_PI) / 2. / ARTIS_PI * 10);
  return (costhetabin * 10) + phibin;
}

__global__ void k_spectra(const Ctx *__restrict__ ctxp, const uint64_t *__restrict__ soa, int64_t n, SpecArgs A) {
  const Ctx &K = *ctxp;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (hi32(soa[PW(n, i, 0)]) != ARTIS_TYPE_ESCAPE) return;
  const uint64_t w32 = soa[PW(n, i, 32)];
  const int escape_type = lo32(w32);
  const int escape_time = hi32(w32);
  const double pos[3] = {asd(soa[PW(n, i, 3)]), asd(soa[PW(n, i, 4)]), asd(soa[PW(n, i, 5)])};
  const double dir[3] = {asd(soa[PW(n, i, 6)]), asd(soa[PW(n, i, 7)]), asd(soa[PW(n, i, 8)])};
  const double e_cmf = asd(soa[PW(n, i, 9)]);
  const double e_rf = asd(soa[PW(n, i, 10)]);
  const double tmin = K.G.tmin, tmax = K.G.tmax;
  const double t_arrive = escape_time - (dot(pos, dir) / ARTIS_CLIGHT_PROP);
  const double cmfcorr = sqrt(1. - (K.G.vmax * K.G.vmax / ARTIS_CLIGHTSQUARED));
  const double t_arrive_cmf = escape_time * cmfcorr;
  if (escape_type == ARTIS_TYPE_GAMMA) {
    if (A.abin != -1) return;
    // add_to_lc_res for the gamma-ray light curve (spectrum.cc:678-680)
    if (t_arrive > tmin && t_arrive < tmax && A.glc) {
      const int nt = spec_timestep(K, A.ntstep, t_arrive);
      if (nt >= 0) unsafeAtomicAdd(&A.glc[nt], e_rf / K.G.ts_width[nt] / A.nprocs);
    }
    if (t_arrive_cmf > tmin && t_arrive_cmf < tmax && A.glccmf) {
      const int nt = spec_timestep(K, A.ntstep, t_arrive_cmf);
      if (nt >= 0) unsafeAtomicAdd(&A.glccmf[nt], e_cmf / K.G.ts_width[nt] / A.nprocs / cmfcorr);
    }
    return;
  }
  if (escape_type != ARTIS_TYPE_RPKT) return;
  if (A.abin >= 0 && escapedirectionbin(dir, A.syn_dir) != A.abin) return;
  const double anglefactor = (A.abin >= 0) ? ARTIS_MABINS : 1.;
  // light_curve.cc:34-62 add_to_lc_res (the direction-bin branch has no cmf light curve)
  if (t_arrive > tmin && t_arrive < tmax && A.lc) {
    const int nt = spec_timestep(K, A.ntstep, t_arrive);
    if (nt >= 0) unsafeAtomicAdd(&A.lc[nt], e_rf / K.G.ts_width[nt] * anglefactor / A.nprocs);
  }
  if (A.abin == -1 && t_arrive_cmf > tmin && t_arrive_cmf < tmax && A.lccmf) {
    const int nt = spec_timestep(K, A.ntstep, t_arrive_cmf);
    if (nt >= 0) unsafeAtomicAdd(&A.lccmf[nt], e_cmf / K.G.ts_width[nt] / A.nprocs / cmfcorr);
  }
  // spectrum.cc:339-452 add_to_spec
  const double nu_rf = asd(soa[PW(n, i, 12)]);
  const double nu_min = K.G.nu_min_r, nu_max = K.G.nu_max_r;
  if (!(t_arrive > tmin && t_arrive < tmax && nu_rf > nu_min && nu_rf < nu_max)) return;
  const int nt = spec_timestep(K, A.ntstep, t_arrive);
  const int nnu = (int)((log(nu_rf) - log(nu_min)) / A.dlognu);
  if (nt < 0 || nnu < 0 || nnu >= A.nnubins) return;
  const double deltaE = e_rf / K.G.ts_width[nt] / A.delta_freq[nnu] / 4.e12 / ARTIS_PI / ARTIS_PARSEC / ARTIS_PARSEC /
                        A.nprocs * anglefactor;
  const double stokes[3] = {asd(soa[PW(n, i, 25)]), asd(soa[PW(n, i, 26)]), asd(soa[PW(n, i, 27)])};
  const int64_t nb = (int64_t)A.ntstep * A.nnubins;
  const int64_t fi = (int64_t)nt * A.nnubins + nnu;
  if (A.flux) unsafeAtomicAdd(&A.flux[fi], deltaE);
  if (A.sflux)
    for (int s = 0; s < 3; s++) unsafeAtomicAdd(&A.sflux[s * nb + fi], stokes[s] * deltaE);
  if (!A.emission) return;
  const uint64_t w13 = soa[PW(n, i, 13)], w19 = soa[PW(n, i, 19)];
  const int nproc = spec_column(A, hi32(w13));
  const int truenproc = spec_column(A, hi32(w19));
  const int64_t ei = fi * A.proccount;
  unsafeAtomicAdd(&A.emission[ei + nproc], deltaE);
  if (A.trueemission) unsafeAtomicAdd(&A.trueemission[ei + truenproc], deltaE);
  if (A.semission)
    for (int s = 0; s < 3; s++) unsafeAtomicAdd(&A.semission[s * nb * A.proccount + ei + nproc], stokes[s] * deltaE);
  const double absorptionfreq = asd(soa[PW(n, i, 21)]);
  const int nnu_abs = (int)((log(absorptionfreq) - log(nu_min)) / A.dlognu);
  const int at = lo32(w19);
  if (nnu_abs >= 0 && nnu_abs < A.nnubins && at >= 0 && A.absorption) {
    const double deltaE_absorption = e_rf / K.G.ts_width[nt] / A.delta_freq[nnu_abs] / 4.e12 / ARTIS_PI /
                                     ARTIS_PARSEC / ARTIS_PARSEC / A.nprocs * anglefactor;
    const int64_t ai = ((int64_t)nt * A.nnubins + nnu_abs) * A.ioncount + A.line_elem[at] * A.maxnions + A.line_ion[at];
    unsafeAtomicAdd(&A.absorption[ai], deltaE_absorption);
    if (A.sabsorption)
      for (int s = 0; s < 3; s++)
        unsafeAtomicAdd(&A.sabsorption[s * nb * A.ioncount + ai], stokes[s] * deltaE_absorption);
  }
}

#endif
