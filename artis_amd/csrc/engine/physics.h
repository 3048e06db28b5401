// physics.h -- device restatement of the reference hot path (one packet per workitem).
//
// Every function cites the reference file:line it follows.  The arithmetic is written in the reference's
// operation order and the engine is compiled with -ffp-contract=off, so that with the same per-packet random
// stream (include/artis_rng.h) a packet's history matches the CPU oracle up to last-bit differences of the
// device libm (exp/log/pow/trig).  Deviations D1-D6 of oracle/oracle.cc apply identically here; the per-cell
// tables of DevCells replace the per-thread cellhistory cache (deviation-free: they are deterministic
// functions of the cell state).
#ifndef ARTIS_PHYSICS_H
#define ARTIS_PHYSICS_H

#include <hip/hip_runtime.h>

#include "artis_constants.h"
#include "artis_rng.h"
#include "engine_dev.h"
#include "packet_soa.h"

#define DEVFN __device__ __forceinline__
#define DEVNI __device__ __noinline__

// error codes written to DevEst::err[0]
enum : int32_t {
  ERR_NONE = 0,
  ERR_UNSUPPORTED_TYPE = 1,
  ERR_SDIST = 2,
  ERR_BADCELL = 3,
  ERR_EDIST = 4,
  ERR_NOEVENT = 5,
  ERR_CONT = 6,
  ERR_MA_RANDOM = 7,
  ERR_MA_SELECT = 8,
  ERR_KPKT = 9,
  ERR_STUCK = 10,
  ERR_LDIST = 11,
  ERR_THICK_MA = 12,
  ERR_NONFINITE = 13,
  ERR_GAMMA = 14,  // an abort() path of the pellet / gamma code (aux = which)
  ERR_VPKT_OVERFLOW = 15,  // the virtual-packet spawn buffer of one event round is full
  ERR_SHELL = 16,  // get_shellcrossdist's consistency checks (boundary.cc:19, 34, 61-62, 95: assert_always)
};

struct __attribute__((aligned(16))) Ctx {
  DevTab T;
  DevGeom G;
  DevCells C;
  DevEst E;
  DevRun R;
  DevVpkt V;
};

// The transport kernels receive the context as a pointer to a device copy (engine.hip: sync_ctx) rather than
// as a by-value kernel argument: the rare-event code is noinline and receives `const Ctx &`, and a reference to a
// by-value kernel argument forces the whole context into per-lane scratch.  Read through that pointer, though,
// every field is a vector load from memory, repeated after any store of the kernel (the compiler cannot prove
// the stores leave the context unchanged): two dependent trips to memory per table access in the hot loops.  So
// each block first copies the context into LDS (CTX_IN_LDS) and works on that copy: a field read is an LDS read.
static_assert(sizeof(Ctx) % 16 == 0, "Ctx is copied in 16-byte chunks");
#define CTX_IN_LDS(ctxp)                                                                  \
  __shared__ Ctx s_ctx_;                                                                  \
  for (int i_ = threadIdx.x; i_ < (int)(sizeof(Ctx) / 16); i_ += blockDim.x)             \
    reinterpret_cast<uint4 *>(&s_ctx_)[i_] = reinterpret_cast<const uint4 *>(ctxp)[i_]; \
  __syncthreads();                                                                        \
  const Ctx &K = s_ctx_;

struct LocalCounters {
  unsigned long long *ctr;   // LDS [35]: 34 reference counters + nesc
  unsigned long long *work;  // LDS [16]
#ifdef ARTIS_STAMPS
  unsigned long long *diag = nullptr;  // diagnostic build: LDS [48] (k_ma)
#endif
};

DEVFN void lctr(const LocalCounters &L, int c) { atomicAdd(&L.ctr[c], 1ull); }
DEVFN void lwork(const LocalCounters &L, int w, unsigned long long v) { atomicAdd(&L.work[w], v); }

DEVFN void fail(const Ctx &K, int code, int pktnumber, int aux) {
  if (atomicCAS(&K.E.err[0], 0, code) == 0) {
    K.E.err[1] = pktnumber;
    K.E.err[2] = aux;
  }
}

// ------------------------------------------------------------------------------------------ atomic data
DEVFN int uion(const Ctx &K, int e, int i) { return K.T.elem_uniqueionoffset[e] + i; }
DEVFN int ulev(const Ctx &K, int e, int i, int l) { return K.T.ion_uniqueleveloffset[uion(K, e, i)] + l; }
DEVFN double epsilon(const Ctx &K, int e, int i, int l) { return K.T.level_epsilon[ulev(K, e, i, l)]; }
DEVFN double stat_weight(const Ctx &K, int e, int i, int l) { return K.T.level_stat_weight[ulev(K, e, i, l)]; }
DEVFN int get_nions(const Ctx &K, int e) { return K.T.elem_nions[e]; }
DEVFN int get_ionstage(const Ctx &K, int e, int i) { return K.T.ion_ionstage[uion(K, e, i)]; }
DEVFN int get_ionisinglevels(const Ctx &K, int e, int i) { return K.T.ion_ionisinglevels[uion(K, e, i)]; }
// atomic.cc:408-422
DEVFN int get_nphixstargets(const Ctx &K, int e, int i, int l) {
  if (i < get_nions(K, e) - 1 && l < get_ionisinglevels(K, e, i)) return K.T.level_nphixstargets[ulev(K, e, i, l)];
  return 0;
}
DEVFN int get_phixsupperlevel(const Ctx &K, int e, int i, int l, int t) {
  return K.T.phixstarget_levelindex[K.T.level_phixstargets_offset[ulev(K, e, i, l)] + t];
}
DEVFN double get_phixsprobability(const Ctx &K, int e, int i, int l, int t) {
  return K.T.phixstarget_probability[K.T.level_phixstargets_offset[ulev(K, e, i, l)] + t];
}
DEVFN double get_phixs_threshold(const Ctx &K, int e, int i, int l, int t) {  // atomic.cc:437-453
  return epsilon(K, e, i + 1, get_phixsupperlevel(K, e, i, l, t)) - epsilon(K, e, i, l);
}
DEVFN const float *level_photoion_xs(const Ctx &K, int e, int i, int l) {
  return K.T.phixs_xs + (int64_t)K.T.level_phixstable[ulev(K, e, i, l)] * K.T.nphixspoints;
}
DEVFN int get_bflutindex(const Ctx &K, int tempindex, int e, int i, int l, int t) {  // sn3d.h:64-69
  return tempindex * K.T.nbf + (-1 - K.T.level_cont_index[ulev(K, e, i, l)] + t);
}
DEVFN int cell_mgi(const Ctx &K, int cellindex) { return K.G.cell_mgi[cellindex]; }

// ------------------------------------------------------------------------------------------ vectors
DEVFN double vec_len(const double x[3]) { return sqrt((x[0] * x[0]) + (x[1] * x[1]) + (x[2] * x[2])); }
DEVFN void vec_norm(const double in[3], double out[3]) {
  const double mag = vec_len(in);
  out[0] = in[0] / mag;
  out[1] = in[1] / mag;
  out[2] = in[2] / mag;
}
DEVFN double dot(const double x[3], const double y[3]) { return (x[0] * y[0]) + (x[1] * y[1]) + (x[2] * y[2]); }
DEVFN void cross_prod(const double v1[3], const double v2[3], double out[3]) {
  out[0] = (v1[1] * v2[2]) - (v2[1] * v1[2]);
  out[1] = (v1[2] * v2[0]) - (v2[2] * v1[0]);
  out[2] = (v1[0] * v2[1]) - (v2[0] * v1[1]);
}
// vectors.h:63-79
DEVFN void angle_ab(const double dir1[3], const double vel[3], double dir2[3]) {
  const double vsqr = dot(vel, vel) / ARTIS_CLIGHTSQUARED;
  const double gamma_rel = 1. / sqrt(1 - vsqr);
  const double ndotv = dot(dir1, vel);
  const double fact1 = gamma_rel * (1 - (ndotv / ARTIS_CLIGHT));
  const double fact2 = (gamma_rel - (gamma_rel * gamma_rel * ndotv / (gamma_rel + 1) / ARTIS_CLIGHT)) / ARTIS_CLIGHT;
  for (int d = 0; d < 3; d++) dir2[d] = (dir1[d] - (vel[d] * fact2)) / fact1;
}
// vectors.h:81-111 with the flow velocity pos/t of vectors.h:37-43
DEVFN double doppler_pos_dir(bool rel, const double pos[3], const double dir[3], double t) {
  const double v[3] = {pos[0] / t, pos[1] / t, pos[2] / t};
  const double ndotv = dot(dir, v);
  double dopplerfactor = 1. - (ndotv / ARTIS_CLIGHT);
  if (rel) {
    const double betasq = dot(v, v) / ARTIS_CLIGHTSQUARED;
    dopplerfactor = dopplerfactor / sqrt(1 - betasq);
  }
  return dopplerfactor;
}
DEVFN double doppler_pos_dir(const Ctx &K, const double pos[3], const double dir[3], double t) {
  return doppler_pos_dir((bool)K.R.relativistic_doppler, pos, dir, t);
}
DEVFN double doppler_packet(const Ctx &K, const Pkt &p) { return doppler_pos_dir(K, p.pos, p.dir, p.prop_time); }
// vectors.h:113-129
DEVFN void move_pkt(const Ctx &K, Pkt &p, double distance) {
  p.pos[0] += (p.dir[0] * distance);
  p.pos[1] += (p.dir[1] * distance);
  p.pos[2] += (p.dir[2] * distance);
  const double dopplerfactor = doppler_packet(K, p);
  p.nu_cmf = p.nu_rf * dopplerfactor;
  p.e_cmf = p.e_rf * dopplerfactor;
}
// vectors.h:131-144
DEVFN void move_pkt_withtime(const Ctx &K, Pkt &p, double distance) {
  const double nu_cmf_old = p.nu_cmf;
  p.prop_time += distance / ARTIS_CLIGHT_PROP;
  move_pkt(K, p, distance);
  if (p.nu_cmf > nu_cmf_old) p.nu_cmf = nu_cmf_old;
}
// vectors.cc:43-58
DEVFN void get_rand_isotropic_unitvec(artis_rng *rng, double out[3]) {
  const double zrand = artis_rng_uniform(rng);
  const double zrand2 = artis_rng_uniform(rng);
  const double mu = -1 + (2. * zrand);
  const double phi = zrand2 * 2 * ARTIS_PI;
  const double sintheta = sqrt(1. - (mu * mu));
  out[0] = sintheta * cos(phi);
  out[1] = sintheta * sin(phi);
  out[2] = mu;
}

// ------------------------------------------------------------------------------------------ rates
DEVFN double dbb(double nu, double T, double W) {  // radfield.h:44-48
  return W * ARTIS_TWOHOVERCLIGHTSQUARED * pow(nu, 3) / expm1(ARTIS_HOVERKB * nu / T);
}
// atomic.cc:87-155
DEVFN double photoionization_crosssection_fromtable(const Ctx &K, const float *xs, double nu_edge, double nu) {
  float sigma_bf;
  if (K.T.phixs_file_version == 1) {
    if (nu == nu_edge) {
      sigma_bf = xs[0];
    } else if (nu <= nu_edge * (1 + K.T.nphixsnuincrement * K.T.nphixspoints)) {
      const int i = (int)floor(nu / (K.T.nphixsnuincrement * nu_edge)) - 10;
      sigma_bf = xs[i];
    } else {
      sigma_bf = xs[K.T.nphixspoints - 1] *
                 pow(nu_edge * (1 + K.T.nphixsnuincrement * K.T.nphixspoints) / nu, 3);
    }
    return sigma_bf;
  }
  const double ireal = (nu / nu_edge - 1.0) / K.T.nphixsnuincrement;
  const int i = (int)floor(ireal);
  if (i < 0) {
    sigma_bf = 0.0;
  } else if (i < K.T.nphixspoints - 1) {
    const double a = xs[i];
    const double b = xs[i + 1];
    const double factor_b = ireal - i;
    sigma_bf = ((1. - factor_b) * a) + (factor_b * b);
  } else {
    const double nu_max_phixs = nu_edge * K.T.last_phixs_nuovernuedge;
    sigma_bf = xs[K.T.nphixspoints - 1] * pow(nu_max_phixs / nu, 3);
  }
  return sigma_bf;
}
// ratecoeff.cc:686-710 (and the identical interpolations ratecoeff.cc:1026-1041, kpkt.cc:69-82)
DEVFN double lut_interp(const Ctx &K, const double *lut, int e, int i, int l, int t, double T) {
  const int lowerindex = (int)floor(log(T / K.T.mintemp) / K.T.T_step_log);
  if (lowerindex < K.T.tablesize - 1) {
    const int upperindex = lowerindex + 1;
    const double T_lower = K.T.mintemp * exp(lowerindex * K.T.T_step_log);
    const double T_upper = K.T.mintemp * exp(upperindex * K.T.T_step_log);
    const double f_upper = lut[get_bflutindex(K, upperindex, e, i, l, t)];
    const double f_lower = lut[get_bflutindex(K, lowerindex, e, i, l, t)];
    return (f_lower + (f_upper - f_lower) / (T_upper - T_lower) * (T - T_lower));
  }
  return lut[get_bflutindex(K, K.T.tablesize - 1, e, i, l, t)];
}
// ltepop.cc:539-556
DEVFN double calculate_sahafact(const Ctx &K, int e, int i, int l, int upperionlevel, double T, double E_threshold) {
  const double g_lower = stat_weight(K, e, i, l);
  const double g_upper = stat_weight(K, e, i + 1, upperionlevel);
  return ARTIS_SAHACONST * g_lower / g_upper * pow(T, -1.5) * exp(E_threshold / ARTIS_KB / T);
}
// macroatom.h:52-105, on the line's values (coll_str_thisline, forbidden, osc_f, P2): col_deexcitation_ratecoeff
// below reads them from the line tables, k_marates from its packed transition items (MaDownItem) -- one expression
DEVFN double col_deexc_core(float T_e, float nne, double epsilon_trans, double coll_str_thisline, bool forbidden,
                            float osc_f, double P2, double lowerstatweight, double upperstatweight) {
  double C = 0.;
  if (coll_str_thisline < 0) {
    if (!forbidden) {
      const double eoverkt = epsilon_trans / (ARTIS_KB * T_e);
      const double g_bar = 0.2;
      const double gauntfac = (eoverkt > 0.33421) ? g_bar : 0.276 * exp(eoverkt) * (-0.5772156649 - log(eoverkt));
      const double g_ratio = lowerstatweight / upperstatweight;
      C = ARTIS_C_0 * 14.51039491 * nne * sqrtf(T_e) * osc_f * P2 * eoverkt * g_ratio * gauntfac;
    } else {
      C = nne * 8.629e-6 * 0.01 * lowerstatweight / sqrtf(T_e);
    }
  } else {
    C = nne * 8.629e-6 * coll_str_thisline / upperstatweight / sqrtf(T_e);
  }
  return C;
}
DEVFN double col_deexcitation_ratecoeff(const Ctx &K, float T_e, float nne, double epsilon_trans, int li,
                                        double lowerstatweight, double upperstatweight) {
  return col_deexc_core(T_e, nne, epsilon_trans, K.T.line_coll[li], K.T.line_forbidden[li] != 0, K.T.line_f[li],
                        K.T.line_ma[li].P2, lowerstatweight, upperstatweight);
}
// col_excitation_ratecoeff's Gaunt factor max(g_bar, 0.276 e^x (-gamma_E - ln x)) is g_bar for every x with
// ln x > -gamma_E = -0.5772 (x > 0.5615): from x > 0.57 on (ln 0.57 = -0.5621) the log is skipped
#define MA_GAUNT_NOLOG 0.57
// macroatom.h:107-150, on the line's values as col_deexc_core
DEVFN double col_exc_core(float T_e, float nne, double coll_strength, bool forbidden, float osc_f, double P2,
                          double epsilon_trans, double lowerstatweight, double upperstatweight) {
  double C = 0.;
  const double eoverkt = epsilon_trans / (ARTIS_KB * T_e);
  if (coll_strength < 0) {
    if (!forbidden) {
      const double g_bar = 0.2;
      const double exp_eoverkt = exp(eoverkt);
      // (above MA_GAUNT_NOLOG the log exceeds -0.5621 > -0.5772: test is negative and Gamma is g_bar whatever its
      // value, so the log is not evaluated -- the same Gamma, bit for bit)
      const double test =
          eoverkt > MA_GAUNT_NOLOG ? -1. : 0.276 * exp_eoverkt * (-0.5772156649 - log(eoverkt));
      const double Gamma = g_bar > test ? g_bar : test;
      C = ARTIS_C_0 * nne * sqrtf(T_e) * 14.51039491 * osc_f * P2 * eoverkt / exp_eoverkt * Gamma;
    } else {
      C = nne * 8.629e-6 * 0.01 * exp(-eoverkt) * upperstatweight / sqrtf(T_e);
    }
  } else {
    C = nne * 8.629e-6 * coll_strength * exp(-eoverkt) / lowerstatweight / sqrtf(T_e);
  }
  return C;
}
DEVFN double col_excitation_ratecoeff(const Ctx &K, float T_e, float nne, int li, double epsilon_trans,
                                      double lowerstatweight, double upperstatweight) {
  return col_exc_core(T_e, nne, K.T.line_coll[li], K.T.line_forbidden[li] != 0, K.T.line_f[li], K.T.line_ma[li].P2,
                      epsilon_trans, lowerstatweight, upperstatweight);
}
// macroatom.h:107-150 col_excitation_ratecoeff on a packed item (TeExcItem, indexed like uptrans_lineindex): the same
// expressions as col_excitation_ratecoeff above on the same values (epsilon_trans = epsilon(upper) - epsilon(level),
// the line's P2, collision strength, oscillator strength and upper statistical weight), from one load per line
DEVFN double te_col_exc(const TeExcItem &it, float T_e, float nne, double lowerstatweight) {
  double C = 0.;
  const double coll_strength = it.coll_str;
  const double eoverkt = it.epsilon_trans / (ARTIS_KB * T_e);
  if (coll_strength < 0) {
    if (!it.forbidden) {
      const double g_bar = 0.2;
      const double exp_eoverkt = exp(eoverkt);
      const double test =
          eoverkt > MA_GAUNT_NOLOG ? -1. : 0.276 * exp_eoverkt * (-0.5772156649 - log(eoverkt));  // (col_exc_core)
      const double Gamma = g_bar > test ? g_bar : test;
      C = ARTIS_C_0 * nne * sqrtf(T_e) * 14.51039491 * it.osc_f * it.P2 * eoverkt / exp_eoverkt * Gamma;
    } else {
      C = nne * 8.629e-6 * 0.01 * exp(-eoverkt) * (double)it.upper_sw / sqrtf(T_e);
    }
  } else {
    C = nne * 8.629e-6 * coll_strength * exp(-eoverkt) / lowerstatweight / sqrtf(T_e);
  }
  return C;
}
// macroatom.cc:503-548 (populations from the per-cell table, B coefficients from LineMA)
DEVFN double rad_deexc_core(double n_u, double n_l, double B_lu, double B_ul, double A_ul, double t_current) {
  double R = 0.0;
  const double tau_sobolev = (B_lu * n_l - B_ul * n_u) * ARTIS_HCLIGHTOVERFOURPI * t_current;
  if (tau_sobolev > 1e-100) {
    const double beta = 1.0 / tau_sobolev * (-expm1(-tau_sobolev));
    R = A_ul * beta;
  }
  return R;
}
DEVFN double rad_deexcitation_ratecoeff_n(const Ctx &K, double n_u, double n_l, int li, double t_current) {
  const LineMA lm = K.T.line_ma[li];
  return rad_deexc_core(n_u, n_l, lm.B_lu, lm.B_ul, K.T.line_A[li], t_current);
}
DEVFN double rad_deexcitation_ratecoeff(const Ctx &K, const double *pops, int e, int i, int upper, int lower,
                                        double epsilon_trans, int li, double t_current) {
  return rad_deexcitation_ratecoeff_n(K, pops[ulev(K, e, i, upper)], pops[ulev(K, e, i, lower)], li, t_current);
}
// radfield.cc:575-600 select_bin: the lowest bin whose upper edge exceeds nu; -2 below the first bin, -1 above
// the last
DEVFN int rf_select_bin(const Ctx &K, double nu) {
  if (nu < K.T.rf_nu_lower_first) return -2;
  int lo = 0, hi = K.T.rf_nbins;  // upper_bound
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (K.T.rf_nu_upper[mid] > nu)
      hi = mid;
    else
      lo = mid + 1;
  }
  return lo >= K.T.rf_nbins ? -1 : lo;
}
// radfield.cc:898-943 radfield(nu, mgi) as the dilute blackbody (T_R, W) it evaluates (radfield.h:44-48): the
// fitted bin's from FIRST_NLTE_RADFIELD_TIMESTEP on under MULTIBIN_RADFIELD_MODEL_ON (false: J_nu = 0, no bin
// or no fit), the cell's full-spectrum one otherwise
DEVFN bool radfield_TW(const Ctx &K, int mgi, double nu, float &T_R, float &W) {
  if (K.R.multibin && K.R.nts >= K.R.first_nlte_rf) {
    const int b = rf_select_bin(K, nu);
    if (b < 0) return false;
    const int64_t mb = (int64_t)mgi * K.T.rf_nbins + b;
    W = K.C.rf_W[mb];
    if (!(W >= 0.f)) return false;
    T_R = K.C.rf_TR[mb];
    return true;
  }
  T_R = K.C.TR[mgi];
  W = K.C.W[mgi];
  return true;
}
DEVFN double radfield_J(const Ctx &K, int mgi, double nu) {
  float T_R, W;
  if (!radfield_TW(K, mgi, nu, T_R, W)) return 0.;
  return dbb(nu, T_R, W);
}
// macroatom.cc:550-643 (J_nu = radfield(nu_trans), radfield.cc:898-943 / radfield.h:44-48, with pow(nu, 3)
// precomputed per line)
DEVFN double rad_exc_core(const Ctx &K, int mgi, double n_u, double n_l, double epsilon_trans, double B_lu, double B_ul,
                          double nu3, double t_current) {
  double R = 0.0;
  const double tau_sobolev = (B_lu * n_l - B_ul * n_u) * ARTIS_HCLIGHTOVERFOURPI * t_current;
  if (tau_sobolev > 1e-100) {
    const double beta = 1.0 / tau_sobolev * (-expm1(-tau_sobolev));
    const double R_over_J_nu = n_l > 0. ? (B_lu - B_ul * n_u / n_l) * beta : B_lu * beta;
    const double nu_trans = epsilon_trans / ARTIS_H;
    float T_R, W;
    if (radfield_TW(K, mgi, nu_trans, T_R, W))
      R = R_over_J_nu * (W * ARTIS_TWOHOVERCLIGHTSQUARED * nu3 / expm1(ARTIS_HOVERKB * nu_trans / T_R));
    else
      R = R_over_J_nu * 0.;
  }
  return R;
}
DEVFN double rad_excitation_ratecoeff_n(const Ctx &K, int mgi, double n_u, double n_l, double epsilon_trans, int li,
                                        double t_current) {
  const LineMA lm = K.T.line_ma[li];
  return rad_exc_core(K, mgi, n_u, n_l, epsilon_trans, lm.B_lu, lm.B_ul, lm.nu3, t_current);
}
DEVFN double rad_excitation_ratecoeff(const Ctx &K, const double *pops, int mgi, int e, int i, int lower, int upper,
                                      double epsilon_trans, int li, double t_current) {
  return rad_excitation_ratecoeff_n(K, mgi, pops[ulev(K, e, i, upper)], pops[ulev(K, e, i, lower)], epsilon_trans, li,
                                    t_current);
}
// macroatom.cc:645-678
DEVFN double rad_recombination_ratecoeff(const Ctx &K, float T_e, float nne, int e, int upperion, int upper, int lower) {
  double R = 0.0;
  const int nt = get_nphixstargets(K, e, upperion - 1, lower);
  for (int t = 0; t < nt; t++) {
    if (get_phixsupperlevel(K, e, upperion - 1, lower, t) == upper) {
      R = nne * lut_interp(K, K.T.spontrecombcoeff, e, upperion - 1, lower, t, T_e);
      break;
    }
  }
  return R;
}
// macroatom.cc:704-743
DEVFN double col_recombination_ratecoeff(const Ctx &K, int mgi, int e, int upperion, int upper, int lower,
                                         double epsilon_trans) {
  const int nt = get_nphixstargets(K, e, upperion - 1, lower);
  for (int t = 0; t < nt; t++) {
    if (get_phixsupperlevel(K, e, upperion - 1, lower, t) == upper) {
      const float nne = K.C.nne[mgi];
      const float T_e = K.C.Te[mgi];
      const double fac1 = epsilon_trans / ARTIS_KB / T_e;
      const int ionstage = get_ionstage(K, e, upperion);
      double g;
      if (ionstage - 1 == 1)
        g = 0.1;
      else if (ionstage - 1 == 2)
        g = 0.2;
      else
        g = 0.3;
      const double sigma_bf =
          (level_photoion_xs(K, e, upperion - 1, lower)[0] * get_phixsprobability(K, e, upperion - 1, lower, t));
      const double sf = calculate_sahafact(K, e, upperion - 1, lower, upper, T_e, epsilon_trans);
      return nne * nne * sf * 1.55e13 * pow((double)T_e, -0.5) * g * sigma_bf * exp(-fac1) / fac1;
    }
  }
  return 0.;
}
// lut_interp's temperature-only part (the bracketing table indices and temperatures) for one T, so that a loop over
// many (level, target) pairs at the same T evaluates its log and exps once: lut_interp_at gives lut_interp's value
// bit for bit (the same expressions on the same arguments)
struct LutT {
  int lowerindex;
  double T_lower, T_upper;
};
DEVFN LutT lut_t(const Ctx &K, double T) {
  LutT r;
  r.lowerindex = (int)floor(log(T / K.T.mintemp) / K.T.T_step_log);
  r.T_lower = r.T_upper = 0.;
  if (r.lowerindex < K.T.tablesize - 1) {
    r.T_lower = K.T.mintemp * exp(r.lowerindex * K.T.T_step_log);
    r.T_upper = K.T.mintemp * exp((r.lowerindex + 1) * K.T.T_step_log);
  }
  return r;
}
DEVFN double lut_interp_at(const Ctx &K, const double *lut, int e, int i, int l, int t, double T, const LutT &lt) {
  if (lt.lowerindex < K.T.tablesize - 1) {
    const double f_upper = lut[get_bflutindex(K, lt.lowerindex + 1, e, i, l, t)];
    const double f_lower = lut[get_bflutindex(K, lt.lowerindex, e, i, l, t)];
    return (f_lower + (f_upper - f_lower) / (lt.T_upper - lt.T_lower) * (T - lt.T_lower));
  }
  return lut[get_bflutindex(K, K.T.tablesize - 1, e, i, l, t)];
}
// macroatom.cc:745-776
DEVFN double col_ionization_ratecoeff(const Ctx &K, float T_e, float nne, int e, int i, int lower, int t,
                                      double epsilon_trans) {
  double g;
  const int ionstage = get_ionstage(K, e, i);
  if (ionstage == 1)
    g = 0.1;
  else if (ionstage == 2)
    g = 0.2;
  else
    g = 0.3;
  const double fac1 = epsilon_trans / ARTIS_KB / T_e;
  const double sigma_bf = level_photoion_xs(K, e, i, lower)[0] * get_phixsprobability(K, e, i, lower, t);
  return nne * 1.55e13 * pow((double)T_e, -0.5) * g * sigma_bf * exp(-fac1) / fac1;
}
// the same with pow(T_e, -0.5) given (rsqrtT), for loops at one T_e
DEVFN double col_ionization_ratecoeff_r(const Ctx &K, float T_e, float nne, int e, int i, int lower, int t,
                                        double epsilon_trans, double rsqrtT) {
  double g;
  const int ionstage = get_ionstage(K, e, i);
  if (ionstage == 1)
    g = 0.1;
  else if (ionstage == 2)
    g = 0.2;
  else
    g = 0.3;
  const double fac1 = epsilon_trans / ARTIS_KB / T_e;
  const double sigma_bf = level_photoion_xs(K, e, i, lower)[0] * get_phixsprobability(K, e, i, lower, t);
  return nne * 1.55e13 * rsqrtT * g * sigma_bf * exp(-fac1) / fac1;
}

// calculate_macroatom_transitionrates (macroatom.cc:57-159): every individual rate of unique level ul in cell mgi,
// in the reference's order -- down transitions, recombination targets, up transitions, photoionisation targets --
// handed to f(kind, j, R, C, epsilon_trans, epsilon_target, epsilon_current); pop(u) is the cell's population of
// unique level u, corrphot(slot) its corrected photoionisation coefficient.  The precompute (k_marates) and the
// exact path of the cached walk both go through here, so their running sums are the same bit for bit.
// f returns true to stop early.
enum { MA_KIND_DOWN = 0, MA_KIND_RECOMB = 1, MA_KIND_UP = 2, MA_KIND_UPHIGHER = 3 };
template <typename Pop, typename Corr, typename F>
DEVFN void ma_foreach_rate(const Ctx &K, int mgi, int ul, double t_mid, Pop pop, Corr corrphot, F f) {
  const int ui = K.T.level_ui[ul];
  const int e = K.T.ion_element[ui];
  const int i = ui - K.T.elem_uniqueionoffset[e];
  const int l = ul - K.T.ion_uniqueleveloffset[ui];
  const float T_e = K.C.Te[mgi];
  const float nne = K.C.nne[mgi];
  const double n_self = pop(ul);
  const double epsilon_current = K.T.level_epsilon[ul];
  const double statweight = K.T.level_stat_weight[ul];
  const int ndowntrans = K.T.level_ndowntrans[ul];
  const int doff = K.T.level_downtrans_offset[ul];
  for (int j = 0; j < ndowntrans; j++) {
    const int li = K.T.downtrans_lineindex[doff + j];
    const int lower = K.T.line_lower[li];
    const double epsilon_target = epsilon(K, e, i, lower);
    const double epsilon_trans = epsilon_current - epsilon_target;
    const double n_l = pop(ul - l + lower);
    const double R = rad_deexcitation_ratecoeff_n(K, n_self, n_l, li, t_mid);
    const double C = col_deexcitation_ratecoeff(K, T_e, nne, epsilon_trans, li, stat_weight(K, e, i, lower), statweight);
    if (f(MA_KIND_DOWN, j, R, C, epsilon_trans, epsilon_target, epsilon_current)) return;
  }
  if (i > 0 && l <= K.T.ion_maxrecombininglevel[ui]) {
    const int nlevels = get_ionisinglevels(K, e, i - 1);
    for (int lower = 0; lower < nlevels; lower++) {
      const double epsilon_target = epsilon(K, e, i - 1, lower);
      const double epsilon_trans = epsilon_current - epsilon_target;
      const double R = rad_recombination_ratecoeff(K, T_e, nne, e, i, l, lower);
      const double C = col_recombination_ratecoeff(K, mgi, e, i, l, lower, epsilon_trans);
      if (f(MA_KIND_RECOMB, lower, R, C, epsilon_trans, epsilon_target, epsilon_current)) return;
    }
  }
  const int nuptrans = K.T.level_nuptrans[ul];
  const int uoff = K.T.level_uptrans_offset[ul];
  for (int j = 0; j < nuptrans; j++) {
    const int li = K.T.uptrans_lineindex[uoff + j];
    const int upper = K.T.line_upper[li];
    const double epsilon_trans = epsilon(K, e, i, upper) - epsilon_current;
    const double n_u = pop(ul - l + upper);
    const double R = rad_excitation_ratecoeff_n(K, mgi, n_u, n_self, epsilon_trans, li, t_mid);
    const double C = col_excitation_ratecoeff(K, T_e, nne, li, epsilon_trans, statweight, stat_weight(K, e, i, upper));
    if (f(MA_KIND_UP, j, R, C, epsilon_trans, 0., epsilon_current)) return;
  }
  if (i < K.T.elem_nions[e] - 1 && l < K.T.ion_ionisinglevels[ui]) {
    const int nt = K.T.level_nphixstargets[ul];
    const int slot0 = K.T.level_phixstargets_offset[ul];
    for (int t = 0; t < nt; t++) {
      const double epsilon_trans = get_phixs_threshold(K, e, i, l, t);
      const double R = corrphot(slot0 + t);
      const double C = col_ionization_ratecoeff(K, T_e, nne, e, i, l, t, epsilon_trans);
      if (f(MA_KIND_UPHIGHER, t, R, C, epsilon_trans, 0., epsilon_current)) return;
    }
  }
}

// ma_foreach_rate for k_marates (the lanes of a wave on one level, so the transition data are wave-uniform): the same
// calls of f with the same values, the down and up transitions read from the packed items (MaDownItem / MaUpItem)
// and software-pipelined -- the item two transitions ahead and the population one ahead are in flight while the
// current rates are evaluated (the plain loop waited on a chain of three dependent loads per transition).  The
// population load is issued before the next item's scalar load: a wait for scalar loads covers all of them.
template <typename Pop, typename Corr, typename F>
DEVFN void ma_foreach_rate_pf(const Ctx &K, int mgi, int ul, double t_mid, Pop pop, Corr corrphot, F f) {
  const int ui = K.T.level_ui[ul];
  const int e = K.T.ion_element[ui];
  const int i = ui - K.T.elem_uniqueionoffset[e];
  const int l = ul - K.T.ion_uniqueleveloffset[ui];
  const int base = ul - l;
  const float T_e = K.C.Te[mgi];
  const float nne = K.C.nne[mgi];
  const double n_self = pop(ul);
  const double epsilon_current = K.T.level_epsilon[ul];
  const double statweight = K.T.level_stat_weight[ul];
  const int ndowntrans = K.T.level_ndowntrans[ul];
  if (ndowntrans > 0) {
    const MaDownItem *DI = K.T.ma_down + K.T.level_downtrans_offset[ul];
    MaDownItem c = DI[0], n1 = DI[ndowntrans > 1 ? 1 : 0];
    double pc = pop(base + c.lower);
    for (int j = 0; j < ndowntrans; j++) {
      const double pn = pop(base + n1.lower);
      const MaDownItem n2 = DI[min(j + 2, ndowntrans - 1)];
      const double epsilon_trans = epsilon_current - c.eps_target;
      const double R = rad_deexc_core(n_self, pc, c.B_lu, c.B_ul, c.A, t_mid);
      const double C = col_deexc_core(T_e, nne, epsilon_trans, c.coll, c.forbidden != 0, c.osc_f, c.P2,
                                      (double)c.lower_sw, statweight);
      if (f(MA_KIND_DOWN, j, R, C, epsilon_trans, c.eps_target, epsilon_current)) return;
      c = n1;
      n1 = n2;
      pc = pn;
    }
  }
  if (i > 0 && l <= K.T.ion_maxrecombininglevel[ui]) {
    const int nlevels = get_ionisinglevels(K, e, i - 1);
    for (int lower = 0; lower < nlevels; lower++) {
      const double epsilon_target = epsilon(K, e, i - 1, lower);
      const double epsilon_trans = epsilon_current - epsilon_target;
      const double R = rad_recombination_ratecoeff(K, T_e, nne, e, i, l, lower);
      const double C = col_recombination_ratecoeff(K, mgi, e, i, l, lower, epsilon_trans);
      if (f(MA_KIND_RECOMB, lower, R, C, epsilon_trans, epsilon_target, epsilon_current)) return;
    }
  }
  const int nuptrans = K.T.level_nuptrans[ul];
  if (nuptrans > 0) {
    const MaUpItem *UI = K.T.ma_up + K.T.level_uptrans_offset[ul];
    MaUpItem c = UI[0], n1 = UI[nuptrans > 1 ? 1 : 0];
    double pc = pop(base + c.upper);
    for (int j = 0; j < nuptrans; j++) {
      const double pn = pop(base + n1.upper);
      const MaUpItem n2 = UI[min(j + 2, nuptrans - 1)];
      const double epsilon_trans = c.eps_upper - epsilon_current;
      const double R = rad_exc_core(K, mgi, pc, n_self, epsilon_trans, c.B_lu, c.B_ul, c.nu3, t_mid);
      const double C = col_exc_core(T_e, nne, c.coll, c.forbidden != 0, c.osc_f, c.P2, epsilon_trans, statweight,
                                    (double)c.upper_sw);
      if (f(MA_KIND_UP, j, R, C, epsilon_trans, 0., epsilon_current)) return;
      c = n1;
      n1 = n2;
      pc = pn;
    }
  }
  if (i < K.T.elem_nions[e] - 1 && l < K.T.ion_ionisinglevels[ui]) {
    const int nt = K.T.level_nphixstargets[ul];
    const int slot0 = K.T.level_phixstargets_offset[ul];
    for (int t = 0; t < nt; t++) {
      const double epsilon_trans = get_phixs_threshold(K, e, i, l, t);
      const double R = corrphot(slot0 + t);
      const double C = col_ionization_ratecoeff(K, T_e, nne, e, i, l, t, epsilon_trans);
      if (f(MA_KIND_UPHIGHER, t, R, C, epsilon_trans, 0., epsilon_current)) return;
    }
  }
}

// The pos-th individual rate of ma_foreach_rate's sequence (pos in [0, nd + nr + nu + nt) of the level's MaMeta),
// with the very expressions of ma_foreach_rate, so that rates evaluated one per lane and summed in order give the
// same sums bit for bit (the wave-parallel exact jump of k_ma_exact)
struct MaItem {
  int kind, j;
  double R, C, et, eg;
};
template <typename Pop, typename Corr>
DEVFN MaItem ma_rate_at(const Ctx &K, int mgi, int ul, double t_mid, int pos, Pop pop, Corr corrphot) {
  const int ui = K.T.level_ui[ul];
  const int e = K.T.ion_element[ui];
  const int i = ui - K.T.elem_uniqueionoffset[e];
  const int l = ul - K.T.ion_uniqueleveloffset[ui];
  const float T_e = K.C.Te[mgi];
  const float nne = K.C.nne[mgi];
  const double epsilon_current = K.T.level_epsilon[ul];
  const double statweight = K.T.level_stat_weight[ul];
  MaItem it;
  const int ndowntrans = K.T.level_ndowntrans[ul];
  // (the down / up transitions from k_marates' packed items: one load before the population, not a chain of three)
  if (pos < ndowntrans) {
    const MaDownItem c = K.T.ma_down[K.T.level_downtrans_offset[ul] + pos];
    const double epsilon_trans = epsilon_current - c.eps_target;
    const double n_self = pop(ul);
    const double n_l = pop(ul - l + c.lower);
    it = {MA_KIND_DOWN, pos, rad_deexc_core(n_self, n_l, c.B_lu, c.B_ul, c.A, t_mid),
          col_deexc_core(T_e, nne, epsilon_trans, c.coll, c.forbidden != 0, c.osc_f, c.P2, (double)c.lower_sw,
                         statweight),
          epsilon_trans, c.eps_target};
    return it;
  }
  pos -= ndowntrans;
  const int nrl = (i > 0 && l <= K.T.ion_maxrecombininglevel[ui]) ? get_ionisinglevels(K, e, i - 1) : 0;
  if (pos < nrl) {
    const int lower = pos;
    const double epsilon_target = epsilon(K, e, i - 1, lower);
    const double epsilon_trans = epsilon_current - epsilon_target;
    it = {MA_KIND_RECOMB, lower, rad_recombination_ratecoeff(K, T_e, nne, e, i, l, lower),
          col_recombination_ratecoeff(K, mgi, e, i, l, lower, epsilon_trans), epsilon_trans, epsilon_target};
    return it;
  }
  pos -= nrl;
  const int nuptrans = K.T.level_nuptrans[ul];
  if (pos < nuptrans) {
    const MaUpItem c = K.T.ma_up[K.T.level_uptrans_offset[ul] + pos];
    const double epsilon_trans = c.eps_upper - epsilon_current;
    const double n_self = pop(ul);
    const double n_u = pop(ul - l + c.upper);
    it = {MA_KIND_UP, pos, rad_exc_core(K, mgi, n_u, n_self, epsilon_trans, c.B_lu, c.B_ul, c.nu3, t_mid),
          col_exc_core(T_e, nne, c.coll, c.forbidden != 0, c.osc_f, c.P2, epsilon_trans, statweight,
                       (double)c.upper_sw),
          epsilon_trans, 0.};
    return it;
  }
  pos -= nuptrans;
  const int t = pos;
  const double epsilon_trans = get_phixs_threshold(K, e, i, l, t);
  it = {MA_KIND_UPHIGHER, t, corrphot(K.T.level_phixstargets_offset[ul] + t),
        col_ionization_ratecoeff(K, T_e, nne, e, i, l, t, epsilon_trans), epsilon_trans, 0.};
  return it;
}

// macroatom.cc:139-146: the INTERNALUPHIGHERNT total of unique level ul (NT_ON; the host's
// nt_ionization_ratecoeff, nonthermal.cc:1684-1712, times epsilon_current)
DEVFN double ma_nt_total(const Ctx &K, int mgi, int ul) {
  if (!K.R.nt_on) return 0.;
  const int ui = K.T.level_ui[ul];
  const int e = K.T.ion_element[ui];
  const int i = ui - K.T.elem_uniqueionoffset[e];
  const int l = ul - K.T.ion_uniqueleveloffset[ui];
  if (!(i < K.T.elem_nions[e] - 1 && l < K.T.ion_ionisinglevels[ui])) return 0.;
  return K.C.nt_Y[(int64_t)mgi * K.T.nions_total + ui] * K.T.level_epsilon[ul];
}
// nonthermal.cc:1640-1655
DEVFN int nt_ionisation_maxupperion(const Ctx &K, int e, int lowerion) {
  const int nions = K.T.elem_nions[e];
  int maxupper = lowerion + 1;
  if (K.R.nt_solve_spencerfano) maxupper = lowerion + 1 + K.R.nt_max_auger;
  if (maxupper > nions - 1) maxupper = nions - 1;
  return maxupper;
}
// nonthermal.cc:1584-1635
DEVFN double nt_ionization_upperion_probability(const Ctx &K, int mgi, int e, int lowerion, int upperion,
                                                bool energyweighted) {
  const int A = K.R.nt_max_auger;
  if (K.R.nt_solve_spencerfano && A > 0) {
    const int numaugerelec = upperion - lowerion - 1;
    const int64_t base = ((int64_t)mgi * K.T.nions_total + uion(K, e, lowerion)) * (A + 1);
    const float *tab = energyweighted ? K.C.nt_ionen : K.C.nt_prob;
    if (numaugerelec < A) return tab[base + numaugerelec];
    if (numaugerelec == A) {
      double prob_remaining = 1.;
      for (int a = 0; a < A; a++) prob_remaining -= tab[base + a];
      return prob_remaining;
    }
    return 0.;
  }
  return (upperion == lowerion + 1) ? 1.0 : 0.;
}
// nonthermal.cc:1657-1682 (a draw that the probabilities do not reach is repeated); -1 if none succeeds
DEVFN int nt_random_upperion(const Ctx &K, artis_rng &rng, int mgi, int e, int lowerion, bool energyweighted) {
  if (K.R.nt_solve_spencerfano && K.R.nt_max_auger > 0) {
    const int maxupper = nt_ionisation_maxupperion(K, e, lowerion);
    for (int attempt = 0; attempt < 1000; attempt++) {
      const double zrand = artis_rng_uniform(&rng);
      double prob_sum = 0.;
      for (int upperion = lowerion + 1; upperion <= maxupper; upperion++) {
        prob_sum += nt_ionization_upperion_probability(K, mgi, e, lowerion, upperion, energyweighted);
        if (zrand <= prob_sum) return upperion;
      }
    }
    return -1;
  }
  return lowerion + 1;
}

// 32-bit key of a running sum v of an action whose total is norm (DevCells::ma_key): round(v / norm * (2^32 - 1)),
// stored as two 16-bit halves (hi in the hot array, lo in the record's second half)
#define MA_KEY_SCALE 4294967295.0
DEVFN uint32_t ma_key32(double v, double norm) {
  if (!(norm > 0.)) return 0u;
  const double q = floor(v / norm * MA_KEY_SCALE + 0.5);
  return (uint32_t)(q < 0. ? 0. : (q > MA_KEY_SCALE ? MA_KEY_SCALE : q));
}
// the same key without the branch (k_mapack's unrolled rows): the quotient is formed for every norm and replaced by
// 0 where ma_key32 returns 0
DEVFN uint32_t ma_key32_nb(double v, double norm) {
  const double q = floor(v / norm * MA_KEY_SCALE + 0.5);
  const double qc = (norm > 0.) ? q : 0.;
  return (uint32_t)(qc < 0. ? 0. : (qc > MA_KEY_SCALE ? MA_KEY_SCALE : qc));
}
// Decides `running sum > x` for x = u * norm (u the uniform draw, q = u * MA_KEY_SCALE) from the key: +1 greater,
// -1 not greater, 0 undecided.  A key is within 0.5 (+ ~1e-5 of rounding in the divisions) of the exact value on
// the 2^32 scale, and q within ~1e-5 of x / norm on that scale.  ma_key_cmp_hi decides from the high half alone
// when it can (the key lies in [hi * 65536, hi * 65536 + 65535]) and returns 2 when the low half is needed.
#define MA_KEY_BAND (0.5 + 1e-4)
DEVFN int ma_key_cmp(uint32_t key, double q) {
  const double d = (double)key - q;
  return d > MA_KEY_BAND ? 1 : (d < -MA_KEY_BAND ? -1 : 0);
}
DEVFN int ma_key_cmp_hi(uint32_t hi, double q) {
  const double d = (double)hi * 65536.0 - q;
  return d > MA_KEY_BAND ? 1 : (d < -(65535.0 + MA_KEY_BAND) ? -1 : 2);
}

// the processrates sums of macroatom.cc:57-159 for one individual rate
DEVFN void ma_accumulate(double pr[ARTIS_MA_ACTION_COUNT], int kind, double R, double C, double epsilon_trans,
                         double epsilon_target, double epsilon_current) {
  if (kind == MA_KIND_DOWN) {
    pr[ARTIS_MA_ACTION_RADDEEXC] += R * epsilon_trans;
    pr[ARTIS_MA_ACTION_COLDEEXC] += C * epsilon_trans;
    pr[ARTIS_MA_ACTION_INTERNALDOWNSAME] += (R + C) * epsilon_target;
  } else if (kind == MA_KIND_RECOMB) {
    pr[ARTIS_MA_ACTION_INTERNALDOWNLOWER] += (R + C) * epsilon_target;
    pr[ARTIS_MA_ACTION_RADRECOMB] += R * epsilon_trans;
    pr[ARTIS_MA_ACTION_COLRECOMB] += C * epsilon_trans;
  } else if (kind == MA_KIND_UP) {
    pr[ARTIS_MA_ACTION_INTERNALUPSAME] += (R + C + 0.) * epsilon_current;
  } else {
    pr[ARTIS_MA_ACTION_INTERNALUPHIGHER] += (R + C) * epsilon_current;
  }
}

#endif
