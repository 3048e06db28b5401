// transport.h -- device r-packet / macro-atom / k-packet propagation (one packet per workitem).
// Restates rpkt.cc, boundary.cc, polarization.cc, vpkt.cc:898-1069, macroatom.cc, kpkt.cc and
// update_packets.cc:137-202 for GRID_UNIFORM, LTE (classic) options; see physics.h for numerics.
#ifndef ARTIS_TRANSPORT_H
#define ARTIS_TRANSPORT_H

#include "physics.h"

// kappa_rpkt_cont of the current step (globals.h:160-170), held in registers
struct Kappa {
  double nu;  // nu_cmf at which it was computed
  double total, es, ff, bf, ffheating;
};

struct Tx {
  const Ctx &K;
  const LocalCounters &L;
  artis_rng rng;
  int nts;
  bool ok;
  unsigned wl = 0, wb = 0;  // diagnostics: lines / bf continua scanned since last reset
  // k_rpkt: the lane's column of the block's line-window image in LDS (16 doubles: nu, then tau coefficients, of
  // 8 consecutive lines; element q at win[q * WAVE_BLOCK]); nullptr: the walk gathers populations itself
  __attribute__((address_space(3))) double *win = nullptr;
  // k_rpkt: the J / nuJ / ffheating terms of the step's estimator segment are left here (est_mgi >= 0) and added
  // after the wave has converged (wave_flush_estimators), so that lanes in the same cell add once per wave
  bool defer_est = false;
  bool vstop = false;  // a virtual-packet spawn found the buffer full (DevVpkt::full): park the packet
  int est_mgi = -1;
  double est_de = 0., est_denu = 0., est_deff = 0.;
  double *est_lds = nullptr;  // k_rpkt: the block's LDS estimator accumulator (DevCells::est_lds_*), or nullptr
  // k_rpkt, models with many bf continua per frequency (the nebular options): the continuum sums of a step are made
  // by the whole wave (wave_kappa_bf before the step, wave_bf_estimators after it) over the wave's 64-slot LDS
  // scratch (coop_d, coop_i), instead of by each lane over its own continua -- lanes at different frequencies
  // reach very different numbers of continua, and the wave waited for its longest list
  double *coop_d = nullptr;
  int *coop_i = nullptr;
  bool pre_on = false;      // kappa_bf of this step precomputed by the wave (pre_kbf; pre_hi: the continua reached)
  double pre_kbf = 0.;
  int pre_hi = 0;
  bool defer_bf = false;    // the detailed-bf estimator terms of the step are left for wave_bf_estimators:
  bool bf_pend = false;     // (cell, frequency, opacity frequency, distance * e_cmf / nu * doppler factor)
  int bf_k = 0, bf_mgi = 0;
  double bf_nu = 0., bf_kapnu = 0., bf_d = 0.;
  // a bound-free absorption's continuum selection (rpkt_event_continuum) is left for the wave (wave_bf_select):
  // (cell, opacity frequency, the draw zrand2 * kappa_bf)
  bool defer_sel = false;
  bool sel_pend = false;
  int sel_k = 0, sel_mgi = 0;
  double sel_nu = 0., sel_rand = 0.;
#ifdef ARTIS_STAMPS
  unsigned long long st[6] = {0, 0, 0, 0, 0, 0}, tlast = 0;  // diagnostic build: cycles per step phase
#endif
  DEVFN Tx(const Ctx &k, const LocalCounters &l) : K(k), L(l), ok(true) {}
  DEVFN void err(int code, int number, int aux) {
    fail(K, code, number, aux);
    ok = false;
  }
};

DEVFN void safeadd(double *p, double v) { unsafeAtomicAdd(p, v); }

// Run a rarely taken noinline step on copies of the packet and the transport state.  A noinline callee needs
// its Pkt& / Tx& in memory; handing it copies keeps the caller's packet and RNG free of address-taking, so
// they stay in registers on the hot path instead of living in scratch.
template <typename F>
DEVFN void cold_call(Tx &x, Pkt &p, F &&f) {
  Tx tx(x.K, x.L);
  tx.rng = x.rng;
  tx.nts = x.nts;
  tx.ok = x.ok;
  Pkt tp = p;
  f(tx, tp);
  p = tp;
  x.rng = tx.rng;
  x.ok = tx.ok;
}

// cold-call policies for do_rpkt_step: the full packet is in registers (megakernel) ...
struct ColdFull {
  template <typename F>
  DEVFN void operator()(Tx &x, Pkt &p, F &&f) const {
    cold_call(x, p, f);
  }
};
// ... or only its hot words are (k_rpkt): the copy is completed from, and written back to, the record in HBM
struct ColdSoa {
  uint64_t *soa;
  int64_t n, idx;
  template <typename F>
  DEVFN void operator()(Tx &x, Pkt &p, F &&f) const {
    Tx tx(x.K, x.L);
    tx.rng = x.rng;
    tx.nts = x.nts;
    tx.ok = x.ok;
    tx.defer_sel = x.defer_sel;
    Pkt tp;
    pkt_copy_hot(tp, p);
    pkt_load_cold(soa, n, idx, tp);
    f(tx, tp);
    pkt_store_cold(soa, n, idx, tp);
    pkt_copy_hot(p, tp);
    x.rng = tx.rng;
    x.ok = tx.ok;
    if (x.defer_sel && tx.sel_pend) {
      x.sel_pend = true;
      x.sel_k = tx.sel_k;
      x.sel_mgi = tx.sel_mgi;
      x.sel_nu = tx.sel_nu;
      x.sel_rand = tx.sel_rand;
    }
  }
};

#ifdef ARTIS_STAMPS
#define STAMP(x, i)                                             \
  do {                                                          \
    const unsigned long long now_ = __builtin_amdgcn_s_memtime(); \
    (x).st[i] += now_ - (x).tlast;                              \
    (x).tlast = now_;                                           \
  } while (0)
#else
#define STAMP(x, i) \
  do {              \
  } while (0)
#endif

// ------------------------------------------------------------------------------------------ emission
// rpkt.cc:975-1025
DEVFN void emitt_rpkt(Tx &x, Pkt &p) {
  p.type = ARTIS_TYPE_RPKT;
  p.last_cross = ARTIS_NONE;
  double dir_cmf[3];
  get_rand_isotropic_unitvec(&x.rng, dir_cmf);
  const double t = -1. * p.prop_time;
  const double vel_vec[3] = {p.pos[0] / t, p.pos[1] / t, p.pos[2] / t};
  angle_ab(dir_cmf, vel_vec, p.dir);
  const double dopplerfactor = doppler_packet(x.K, p);
  p.nu_rf = p.nu_cmf / dopplerfactor;
  p.e_rf = p.e_cmf / dopplerfactor;
  p.stokes[0] = 1.;
  p.stokes[1] = 0.;
  p.stokes[2] = 0.;
  double dummy_dir[3] = {0., 0., 1.};
  cross_prod(p.dir, dummy_dir, p.pol_dir);
  if ((dot(p.pol_dir, p.pol_dir)) < 1.e-8) {
    dummy_dir[0] = dummy_dir[2] = 0.0;
    dummy_dir[1] = 1.0;
    cross_prod(p.dir, dummy_dir, p.pol_dir);
  }
  vec_norm(p.pol_dir, p.pol_dir);
}

// vpkt.cc:898-929
DEVFN double rot_angle(const double n1[3], const double n2[3], const double ref1[3], const double ref2[3]) {
  double i = 0;
  double ref1_sc[3];
  ref1_sc[0] = n1[0] * dot(n1, n2) - n2[0];
  ref1_sc[1] = n1[1] * dot(n1, n2) - n2[1];
  ref1_sc[2] = n1[2] * dot(n1, n2) - n2[2];
  vec_norm(ref1_sc, ref1_sc);
  double c1 = dot(ref1_sc, ref1);
  const double c2 = dot(ref1_sc, ref2);
  if (c1 < -1) c1 = -1;
  if (c1 > 1) c1 = 1;
  if ((c1 > 0) && (c2 > 0)) i = acos(c1);
  if ((c1 > 0) && (c2 < 0)) i = 2 * acos(-1.) - acos(c1);
  if ((c1 < 0) && (c2 < 0)) i = acos(-1.) + acos(fabs(c1));
  if ((c1 < 0) && (c2 > 0)) i = acos(-1.) - acos(fabs(c1));
  if (c1 == 0) i = acos(-1.) / 2.;
  if (c2 == 0) i = 0.0;
  return i;
}
// vpkt.cc:932-944
DEVFN void meridian(const double n[3], double ref1[3], double ref2[3]) {
  ref1[0] = -1. * n[0] * n[2] / sqrt(n[0] * n[0] + n[1] * n[1]);
  ref1[1] = -1. * n[1] * n[2] / sqrt(n[0] * n[0] + n[1] * n[1]);
  ref1[2] = (1 - (n[2] * n[2])) / sqrt(n[0] * n[0] + n[1] * n[1]);
  ref2[0] = n[2] * ref1[1] - n[1] * ref1[2];
  ref2[1] = n[0] * ref1[2] - n[2] * ref1[0];
  ref2[2] = n[1] * ref1[0] - n[0] * ref1[1];
}
// vpkt.cc:1022-1069 (only the E-field result is used)
DEVFN void lorentz(const double e_rf[3], const double n_rf[3], const double v[3], double e_cmf[3]) {
  double beta[3], e_par[3], e_perp[3], b_rf[3], v_cr_b[3];
  beta[0] = v[0] / ARTIS_CLIGHT;
  beta[1] = v[1] / ARTIS_CLIGHT;
  beta[2] = v[2] / ARTIS_CLIGHT;
  const double vsqr = dot(beta, beta);
  const double gamma_rel = 1. / (sqrt(1 - vsqr));
  const double edb = (e_rf[0] * beta[0] + e_rf[1] * beta[1] + e_rf[2] * beta[2]);
  e_par[0] = edb * beta[0] / (vsqr);
  e_par[1] = edb * beta[1] / (vsqr);
  e_par[2] = edb * beta[2] / (vsqr);
  e_perp[0] = e_rf[0] - e_par[0];
  e_perp[1] = e_rf[1] - e_par[1];
  e_perp[2] = e_rf[2] - e_par[2];
  b_rf[0] = n_rf[1] * e_rf[2] - n_rf[2] * e_rf[1];
  b_rf[1] = n_rf[2] * e_rf[0] - n_rf[0] * e_rf[2];
  b_rf[2] = n_rf[0] * e_rf[1] - n_rf[1] * e_rf[0];
  v_cr_b[0] = beta[1] * b_rf[2] - beta[2] * b_rf[1];
  v_cr_b[1] = beta[2] * b_rf[0] - beta[0] * b_rf[2];
  v_cr_b[2] = beta[0] * b_rf[1] - beta[1] * b_rf[0];
  e_cmf[0] = e_par[0] + gamma_rel * (e_perp[0] + v_cr_b[0]);
  e_cmf[1] = e_par[1] + gamma_rel * (e_perp[1] + v_cr_b[1]);
  e_cmf[2] = e_par[2] + gamma_rel * (e_perp[2] + v_cr_b[2]);
  vec_norm(e_cmf, e_cmf);
}
// vpkt.cc:947-1019
DEVFN void frame_transform(const double n_rf[3], double *Q, double *U, const double v[3], double n_cmf[3]) {
  double ref1[3], ref2[3], e_rf[3], e_cmf[3];
  double theta_rot = 0.;
  meridian(n_rf, ref1, ref2);
  const double Q0 = *Q;
  const double U0 = *U;
  const double p = sqrt(Q0 * Q0 + U0 * U0);
  double ra = 0;
  if (p > 0) {
    const double c2 = Q0 / p;
    const double s2 = U0 / p;
    if ((c2 > 0) && (s2 > 0)) ra = acos(Q0 / p) / 2.;
    if ((c2 < 0) && (s2 > 0)) ra = (acos(-1.) - acos(fabs(Q0 / p))) / 2.;
    if ((c2 < 0) && (s2 < 0)) ra = (acos(-1.) + acos(fabs(Q0 / p))) / 2.;
    if ((c2 > 0) && (s2 < 0)) ra = (2. * acos(-1.) - acos(fabs(Q0 / p))) / 2.;
    if (c2 == 0) {
      ra = 0.25 * acos(-1.);
      if (U0 < 0) ra = 0.75 * acos(-1.);
    }
    if (s2 == 0) {
      ra = 0.0;
      if (Q0 < 0) ra = 0.5 * acos(-1.);
    }
  }
  e_rf[0] = cos(ra) * ref1[0] - sin(ra) * ref2[0];
  e_rf[1] = cos(ra) * ref1[1] - sin(ra) * ref2[1];
  e_rf[2] = cos(ra) * ref1[2] - sin(ra) * ref2[2];
  angle_ab(n_rf, v, n_cmf);
  lorentz(e_rf, n_rf, v, e_cmf);
  meridian(n_cmf, ref1, ref2);
  const double r1 = e_cmf[0] * ref1[0] + e_cmf[1] * ref1[1] + e_cmf[2] * ref1[2];
  const double r2 = e_cmf[0] * ref2[0] + e_cmf[1] * ref2[1] + e_cmf[2] * ref2[2];
  if ((r1 > 0) && (r2 < 0)) theta_rot = acos(r1);
  if ((r1 < 0) && (r2 < 0)) theta_rot = acos(-1.) - acos(fabs(r1));
  if ((r1 < 0) && (r2 > 0)) theta_rot = acos(-1.) + acos(fabs(r1));
  if ((r1 > 0) && (r2 > 0)) theta_rot = 2 * acos(-1.) - acos(r1);
  if (r1 == 0) theta_rot = acos(-1.) / 2.;
  if (r2 == 0) theta_rot = 0.0;
  if (r1 > 1) theta_rot = 0.0;
  if (r1 < -1) theta_rot = acos(-1.);
  *Q = cos(2 * theta_rot) * p;
  *U = sin(2 * theta_rot) * p;
}
// polarization.cc:6-157
DEVNI void escat_rpkt(Tx &x, Pkt &p) {
  p.type = ARTIS_TYPE_RPKT;
  p.last_cross = ARTIS_NONE;
  const double t = p.prop_time;
  const double vel_vec[3] = {p.pos[0] / t, p.pos[1] / t, p.pos[2] / t};
  double Qi = p.stokes[1];
  double Ui = p.stokes[2];
  double old_dir_cmf[3];
  frame_transform(p.dir, &Qi, &Ui, vel_vec, old_dir_cmf);
  double M = 0., mu = 0., phisc = 0.;
  if (x.K.R.pol_dipole) {
    double pr = 0., xx = 0.;
    int tries = 0;
    do {
      const double zrand = artis_rng_uniform(&x.rng);
      const double zrand2 = artis_rng_uniform(&x.rng);
      const double zrand3 = artis_rng_uniform(&x.rng);
      M = 2 * zrand - 1;
      mu = pow(M, 2.);
      phisc = 2 * ARTIS_PI * zrand2;
      pr = (mu + 1) + (mu - 1) * (cos(2 * phisc) * Qi + sin(2 * phisc) * Ui);
      xx = 2 * zrand3;
      if (++tries > 1000000) {
        x.err(ERR_STUCK, p.number, 1);
        return;
      }
    } while (xx > pr);
  } else {
    const double zrand = artis_rng_uniform(&x.rng);
    const double zrand2 = artis_rng_uniform(&x.rng);
    M = 2. * zrand - 1;
    mu = pow(M, 2.);
    phisc = 2 * ARTIS_PI * zrand2;
  }
  const double tsc = acos(M);
  double nd[3];
  const double *od = old_dir_cmf;
  if (fabs(od[2]) < 0.99999) {
    nd[0] = sin(tsc) / sqrt(1. - pow(od[2], 2.)) * (od[1] * sin(phisc) - od[0] * od[2] * cos(phisc)) + od[0] * cos(tsc);
    nd[1] = sin(tsc) / sqrt(1 - pow(od[2], 2.)) * (-od[0] * sin(phisc) - od[1] * od[2] * cos(phisc)) + od[1] * cos(tsc);
    nd[2] = sin(tsc) * cos(phisc) * sqrt(1 - pow(od[2], 2.)) + od[2] * cos(tsc);
  } else {
    nd[0] = sin(tsc) * cos(phisc);
    nd[1] = sin(tsc) * sin(phisc);
    nd[2] = (od[2] > 0) ? cos(tsc) : -cos(tsc);
  }
  double ref1[3], ref2[3];
  meridian(od, ref1, ref2);
  const double i1 = rot_angle(od, nd, ref1, ref2);
  const double cos2i1 = cos(2 * i1);
  const double sin2i1 = sin(2 * i1);
  const double Qold = Qi * cos2i1 - Ui * sin2i1;
  const double Uold = Qi * sin2i1 + Ui * cos2i1;
  mu = dot(od, nd);
  const double Inew = 0.75 * ((mu * mu + 1.0) + Qold * (mu * mu - 1.0));
  double Qnew = 0.75 * ((mu * mu - 1.0) + Qold * (mu * mu + 1.0));
  double Unew = 1.5 * mu * Uold;
  Qnew = Qnew / Inew;
  Unew = Unew / Inew;
  meridian(nd, ref1, ref2);
  const double i2 = ARTIS_PI + rot_angle(nd, od, ref1, ref2);
  const double cos2i2 = cos(2 * i2);
  const double sin2i2 = sin(2 * i2);
  double Q = Qnew * cos2i2 + Unew * sin2i2;
  double U = -Qnew * sin2i2 + Unew * cos2i2;
  const double vel_rev[3] = {-vel_vec[0], -vel_vec[1], -vel_vec[2]};
  double dummy_dir[3];
  frame_transform(nd, &Q, &U, vel_rev, dummy_dir);
  p.stokes[0] = 1.0;
  p.stokes[1] = Q;
  p.stokes[2] = U;
  p.dir[0] = dummy_dir[0];
  p.dir[1] = dummy_dir[1];
  p.dir[2] = dummy_dir[2];
  const double dopplerfactor = doppler_packet(x.K, p);
  p.nu_rf = p.nu_cmf / dopplerfactor;
  p.e_rf = p.e_cmf / dopplerfactor;
}

// ------------------------------------------------------------------------------------------ boundary
// boundary.cc:14-99 get_shellcrossdist: the closest forward distance of the ray to an expanding spherical shell, -1
// without a forward intersection (or a tangential one).  The reference's assert_always checks set *bad (-> ERR_SHELL).
DEVFN double get_shellcrossdist(const double pos[3], const double dir[3], const double shellradius,
                                const bool isinnerboundary, const double tstart, bool *bad) {
  if (!(shellradius > 0)) *bad = true;
  const double speed = vec_len(dir) * ARTIS_CLIGHT_PROP;
  const double a = dot(dir, dir) - pow(shellradius / tstart / speed, 2);
  const double b = 2 * (dot(dir, pos) - pow(shellradius, 2) / tstart / speed);
  const double c = dot(pos, pos) - pow(shellradius, 2);
  const double discriminant = pow(b, 2) - 4 * a * c;
  if (discriminant < 0) {
    if (!(shellradius < vec_len(pos))) *bad = true;
    return -1;
  }
  if (discriminant > 0) {
    double d1 = (-b + sqrt(discriminant)) / 2 / a;
    double d2 = (-b - sqrt(discriminant)) / 2 / a;
    double posfinal1[3], posfinal2[3];
    for (int d = 0; d < 3; d++) {  // cblas_dcopy + cblas_daxpy
      posfinal1[d] = pos[d] + d1 * dir[d];
      posfinal2[d] = pos[d] + d2 * dir[d];
    }
    const double shellradiusfinal1 = shellradius / tstart * (tstart + d1 / speed);
    const double shellradiusfinal2 = shellradius / tstart * (tstart + d2 / speed);
    if (!(fabs(vec_len(posfinal1) / shellradiusfinal1 - 1.) < 1e-3)) *bad = true;
    if (!(fabs(vec_len(posfinal2) / shellradiusfinal2 - 1.) < 1e-3)) *bad = true;
    // solutions that would enter the boundary from the wrong radial direction do not count
    if (isinnerboundary) {
      if (dot(posfinal1, dir) > 0.) d1 = -1;
      if (dot(posfinal2, dir) > 0.) d2 = -1;
    } else {
      if (dot(posfinal1, dir) < 0.) d1 = -1;
      if (dot(posfinal2, dir) < 0.) d2 = -1;
    }
    if (d1 < 0 && d2 < 0) return -1;
    if (d2 < 0) return d1;
    if (d1 < 0) return d2;
    return fmin(d1, d2);
  }
  // exactly one (tangential) intersection: ignored
  if (!(shellradius <= vec_len(pos))) *bad = true;
  return -1.;
}

// boundary.cc:101-330, GRID_SPHERICAL1D: the radial coordinate and the two expanding shells of the cell
DEVFN double boundary_cross_sph(const Ctx &K, Pkt &p, int *snext, bool *bad) {
  const double tstart = p.prop_time;
  const int cellindex = p.where;
  const double tmin = K.G.tmin;
  const int n0 = K.G.ncoordgrid[0];
  const double initpos = vec_len(p.pos);
  const double cmin = K.G.cell_pos_min[(int64_t)cellindex * 3];
  const double cmax = cmin + K.G.cell_wid[cellindex];  // get_cellcoordmax: pos_min + wid_init(cellindex)
  const double vel = dot(p.pos, p.dir) / vec_len(p.pos) * ARTIS_CLIGHT_PROP;  // radial velocity
  int last_cross = p.last_cross;
  for (int flip = 0; flip < 2; flip++) {
    const int direction = flip ? ARTIS_POS_X : ARTIS_NEG_X;
    const int invdirection = !flip ? ARTIS_POS_X : ARTIS_NEG_X;
    const int cellindexstride = flip ? -1 : 1;
    bool outside;
    if (flip)
      outside = initpos < (cmin / tmin * tstart - 10.);
    else
      outside = initpos > (cmax / tmin * tstart + 10.);
    if (outside && (last_cross != direction)) {
      if ((vel - (initpos / tstart)) > 0) {
        if ((cellindex == (n0 - 1) && cellindexstride > 0) || (cellindex == 0 && cellindexstride < 0)) {
          *snext = -99;
          return 0;
        }
        *snext = p.where + cellindexstride;
        p.last_cross = invdirection;
        return 0;
      }
      last_cross = direction;
    }
  }
  last_cross = ARTIS_NONE;  // the shell distances below exclude the wrong radial directions themselves
  const double r_inner = cmin * tstart / tmin;
  const double d_inner = (r_inner > 0.) ? get_shellcrossdist(p.pos, p.dir, r_inner, true, tstart, bad) : -1.;
  const double tminb = d_inner / ARTIS_CLIGHT_PROP;
  const double r_outer = cmax * tstart / tmin;
  const double d_outer = get_shellcrossdist(p.pos, p.dir, r_outer, false, tstart, bad);
  const double tmaxb = d_outer / ARTIS_CLIGHT_PROP;
  double time = 1.e99;
  if ((tmaxb > 0) && (tmaxb < time) && (last_cross != ARTIS_NEG_X)) {
    time = tmaxb;
    if (cellindex == (n0 - 1)) {
      *snext = -99;
    } else {
      *snext = p.where + 1;
      p.last_cross = ARTIS_POS_X;
    }
  }
  if ((tminb > 0) && (tminb < time) && (last_cross != ARTIS_POS_X)) {
    time = tminb;
    if (cellindex == 0) {
      *snext = -99;
    } else {
      *snext = p.where - 1;
      p.last_cross = ARTIS_NEG_X;
    }
  }
  return ARTIS_CLIGHT_PROP * time;
}

// rpkt.cc:659-661, gammapkt.cc:551-553: the largest plausible boundary distance of a step
DEVFN double max_sdist(const Ctx &K, const Pkt &p, double sdist) {
  return K.G.spherical ? 2 * K.G.rmax * (p.prop_time + sdist / ARTIS_CLIGHT_PROP) / K.G.tmin
                       : K.G.rmax * p.prop_time / K.G.tmin;
}

// boundary.cc:101-330 (GRID_UNIFORM; GRID_SPHERICAL1D in boundary_cross_sph)
DEVFN double boundary_cross(Tx &x, Pkt &p, int *snext) {
  const Ctx &K = x.K;
  if (__builtin_expect(__builtin_amdgcn_readfirstlane(K.G.spherical), 0)) {
    bool bad = false;
    const double d = boundary_cross_sph(K, p, snext, &bad);
    if (bad) x.err(ERR_SHELL, p.number, p.where);
    return d;
  }
  const double tstart = p.prop_time;
  const int cellindex = p.where;
  const double tmin = K.G.tmin;
  const int n0 = K.G.ncoordgrid[0], n1 = K.G.ncoordgrid[1], n2 = K.G.ncoordgrid[2];
  const int n[3] = {n0, n1, n2};
  const int stride[3] = {1, n0, n0 * n1};
  double initpos[3], cmax[3], cmin[3], vel[3];
  for (int d = 0; d < 3; d++) {
    initpos[d] = p.pos[d];
    cmin[d] = K.G.cell_pos_min[(int64_t)cellindex * 3 + d];
    cmax[d] = cmin[d] + K.G.wid;
    vel[d] = p.dir[d] * ARTIS_CLIGHT_PROP;
  }
  const int pointnum[3] = {cellindex % n0, (cellindex / n0) % n1, (cellindex / (n0 * n1)) % n2};
  int last_cross = p.last_cross;
  const int negd[3] = {ARTIS_NEG_X, ARTIS_NEG_Y, ARTIS_NEG_Z};
  const int posd[3] = {ARTIS_POS_X, ARTIS_POS_Y, ARTIS_POS_Z};
  for (int d = 0; d < 3; d++) {
    for (int flip = 0; flip < 2; flip++) {
      const int direction = flip ? posd[d] : negd[d];
      const int invdirection = !flip ? posd[d] : negd[d];
      const int cellindexstride = flip ? -stride[d] : stride[d];
      bool outside;
      if (flip)
        outside = initpos[d] < (cmin[d] / tmin * tstart - 10.);
      else
        outside = initpos[d] > (cmax[d] / tmin * tstart + 10.);
      if (outside && (last_cross != direction)) {
        if ((vel[d] - (initpos[d] / tstart)) > 0) {
          if ((pointnum[d] == (n[d] - 1) && cellindexstride > 0) || (pointnum[d] == 0 && cellindexstride < 0)) {
            *snext = -99;
            return 0;
          }
          *snext = p.where + cellindexstride;
          p.last_cross = invdirection;
          return 0;
        }
        last_cross = direction;
      }
    }
  }
  double tmaxb[3], tminb[3];
  for (int d = 0; d < 3; d++) {
    tmaxb[d] = ((initpos[d] - (vel[d] * tstart)) / ((cmax[d]) - (vel[d] * tmin)) * tmin) - tstart;
    tminb[d] = ((initpos[d] - (vel[d] * tstart)) / ((cmin[d]) - (vel[d] * tmin)) * tmin) - tstart;
  }
  double time = 1.e99;
  for (int d = 0; d < 3; d++) {
    if ((tmaxb[d] > 0) && (tmaxb[d] < time) && (last_cross != negd[d])) {
      time = tmaxb[d];
      if (pointnum[d] == (n[d] - 1)) {
        *snext = -99;
      } else {
        *snext = p.where + stride[d];
        p.last_cross = posd[d];
      }
    }
    if ((tminb[d] > 0) && (tminb[d] < time) && (last_cross != posd[d])) {
      time = tminb[d];
      if (pointnum[d] == 0) {
        *snext = -99;
      } else {
        *snext = p.where - stride[d];
        p.last_cross = negd[d];
      }
    }
  }
  return ARTIS_CLIGHT_PROP * time;
}
// boundary.cc:332-357
DEVFN void change_cell(Tx &x, Pkt &p, int snext) {
  if (snext == -99) {
    p.escape_type = p.type;
    p.escape_time = (int)p.prop_time;
    p.type = ARTIS_TYPE_ESCAPE;
    lctr(x.L, 34);  // nesc
  } else {
    p.where = snext;
    lctr(x.L, CTR_CELLCROSSINGS);
  }
}

// ------------------------------------------------------------------------------------------ opacity
// rpkt.cc:1075-1207: one continuum's contribution sigma*prob*corr (returns false if not included / inactive).
// The cell's data come from its DevCells::bfcell row (n_level, or 0 when the inclusion rule of rpkt.cc:1116-1118
// excludes the continuum, and the departure ratio), the continuum's from DevTab::bfc; `expfac` is
// exp(-HOVERKB * nu / T_e), which the reference evaluates per continuum with the same arguments (BfCell::expfac).
struct BfCell {
  const double2 *row;  // DevCells::bfcell + k * nbf
  double expfac;
};
DEVFN BfCell bf_cell(const Ctx &K, int k, int mgi, double nu) {
  const double T_e = K.C.Te[mgi];
  return BfCell{K.C.bfcell + (int64_t)k * K.T.nbf, exp(-ARTIS_HOVERKB * nu / T_e)};
}
DEVFN bool bf_contribution(const Ctx &K, const BfCell &cell, int i, double nu, double *nnlevel_out,
                           double *gcontr_out) {
  const BfCont c = K.T.bfc[i];
  const double2 cb = cell.row[i];
  const double nnlevel = cb.x;
  if (!(nu <= c.nu_max && nnlevel > 0)) return false;
  const double sigma_bf = photoionization_crosssection_fromtable(K, K.T.phixs_xs + c.xs_off, c.nu_edge, nu);
  const double stimfactor = cb.y * cell.expfac;
  double corrfactor = 1 - stimfactor;
  if (corrfactor < 0) corrfactor = 0.;
  *nnlevel_out = nnlevel;
  *gcontr_out = sigma_bf * c.probability * corrfactor;
  return true;
}
// bf_contribution of U continua at once (the wave's item loops), staged so that the table loads of the U items are in
// flight together: the records, then both cross-section points (indices clamped into the table; a value the
// branch taken does not use is discarded).  The expressions are bf_contribution's and
// photoionization_crosssection_fromtable's (version-2 tables; version 1 goes through the scalar function).
template <int U>
DEVFN void bf_contribution_batch(const Ctx &K, const BfCell (&cell)[U], const int (&ci)[U], const double (&nu)[U],
                                 bool (&ok)[U], double (&nn)[U], double (&gc)[U]) {
  if (K.T.phixs_file_version == 1) {
#pragma unroll
    for (int u = 0; u < U; u++) ok[u] = bf_contribution(K, cell[u], ci[u], nu[u], &nn[u], &gc[u]);
    return;
  }
  BfCont c[U];
  double2 cb[U];
#pragma unroll
  for (int u = 0; u < U; u++) {
    c[u] = K.T.bfc[ci[u]];
    cb[u] = cell[u].row[ci[u]];
  }
  const int np = K.T.nphixspoints;
  double ireal[U];
  int ix[U];
  float xa[U], xb[U];
#pragma unroll
  for (int u = 0; u < U; u++) {
    ireal[u] = (nu[u] / c[u].nu_edge - 1.0) / K.T.nphixsnuincrement;
    ix[u] = (int)floor(ireal[u]);
    const int la = ix[u] < 0 ? 0 : (ix[u] < np - 1 ? ix[u] : np - 1);
    const float *xs = K.T.phixs_xs + max(c[u].xs_off, 0);
    xa[u] = xs[la];
    xb[u] = xs[min(la + 1, np - 1)];
  }
#pragma unroll
  for (int u = 0; u < U; u++) {
    ok[u] = nu[u] <= c[u].nu_max && cb[u].x > 0;
    float sigma;
    if (ix[u] < 0) {
      sigma = 0.0;
    } else if (ix[u] < np - 1) {
      const double a = xa[u], b = xb[u];
      const double factor_b = ireal[u] - ix[u];
      sigma = ((1. - factor_b) * a) + (factor_b * b);
    } else {
      const double nu_max_phixs = c[u].nu_edge * K.T.last_phixs_nuovernuedge;
      sigma = xa[u] * pow(nu_max_phixs / nu[u], 3);
    }
    const double sigma_bf = sigma;
    const double stimfactor = cb[u].y * cell[u].expfac;
    double corrfactor = 1 - stimfactor;
    if (corrfactor < 0) corrfactor = 0.;
    nn[u] = cb[u].x;
    gc[u] = sigma_bf * c[u].probability * corrfactor;
  }
}
// The continua a frequency reaches: hi = the reference's loop length (it breaks at the first continuum with
// nu < nu_edge, the edges ascending), lo = the first continuum whose cross-section table still covers nu
// (nu <= nu_edge * last_phixs_nuovernuedge, ascending with the edges): below lo, bf_contribution is false (and the
// detailed-bf window test fails), so the sums over [lo, hi) are the reference's sums over [0, hi).  Two binary
// searches over DevTab::bf_edge2 (nu_edge, nu_max), a fixed number of steps (no divergence between lanes).
DEVFN void bf_range(const Ctx &K, double nu, int &lo, int &hi) {
  const double2 *e = K.T.bf_edge2;
  const int nb = K.T.nbf;
  // hi: the first continuum with nu < nu_edge (nb if none); lo: the first with nu <= nu_max, at most hi.  Below
  // the lowest edge both are 0 (one load instead of the search's chain of dependent ones: the virtual packets of
  // config 5 and every r-packet redward of the continua)
  if (nb == 0 || nu < e[0].x) {
    lo = hi = 0;
    return;
  }
  int h = 0, l = 0;
  for (int step = nb > 0 ? 1 << (31 - __clz(nb)) : 0; step > 0; step >>= 1) {
    if (h + step <= nb && !(nu < e[h + step - 1].x)) h += step;
    if (l + step <= nb && nu > e[l + step - 1].y) l += step;
  }
  hi = h;
  lo = min(l, h);
}
// rpkt.cc:1075-1207 calculate_kappa_bf_gammacontr: the kappa_bf total (the cumulative array is re-scanned on demand)
DEVFN double kappa_bf_total(Tx &x, int k, int mgi, double nu) {
  const Ctx &K = x.K;
  if (x.pre_on) {  // made by the wave before the step (wave_kappa_bf): the same sum in the same order
    x.pre_on = false;
    lwork(x.L, WK_BF_ACTIVE, (unsigned long long)x.pre_hi);
    x.wb += (unsigned)x.pre_hi;
    return x.pre_kbf;
  }
  double kappa_bf_sum = 0.;
  int lo, hi;
  bf_range(K, nu, lo, hi);
  const unsigned long long nactive = (unsigned)hi;  // (the continua the reference's loop visits)
  const BfCell cell = bf_cell(K, k, mgi, nu);
  for (int i = lo; i < hi; i++) {
    double nnlevel, gc;
    if (bf_contribution(K, cell, i, nu, &nnlevel, &gc)) kappa_bf_sum += nnlevel * gc;
  }
  lwork(x.L, WK_BF_ACTIVE, nactive);
  x.wb += (unsigned)nactive;
  return kappa_bf_sum;
}
// rpkt.cc:1209-1295 (deviation D2: always recomputed)
DEVFN void calculate_kappa_rpkt_cont(Tx &x, const Pkt &p, int k, int mgi, Kappa &kap) {
  const Ctx &K = x.K;
  const double nu_cmf = p.nu_cmf;
  const float nne = K.C.nne[mgi];
  double sigma = 0.0, kappa_ff = 0., kappa_bf = 0., kappa_ffheating = 0.;
  lwork(x.L, WK_KAPPA_EVALS, 1);
  if (K.R.do_r_lc) {
    const float T_e = K.C.Te[mgi];
    const double ffsum = K.C.ffsum[k];
    const double ff = ffsum * (3.69255e8 / sqrt((double)T_e) * pow(nu_cmf, -3) * nne *
                               (1 - exp(-ARTIS_HOVERKB * nu_cmf / T_e)));  // rpkt.cc:1061
    if (K.R.opacity_case == 4) {
      sigma = ARTIS_SIGMA_T * nne;
      kappa_ff = ff;
      kappa_ffheating = kappa_ff;
      kappa_bf = kappa_bf_total(x, k, mgi, nu_cmf);
    } else {
      kappa_ff = 1e5 * ff;
    }
  }
  kap.nu = nu_cmf;
  kap.total = sigma + kappa_bf + kappa_ff;
  kap.es = sigma;
  kap.ff = kappa_ff;
  kap.bf = kappa_bf;
  kap.ffheating = kappa_ffheating;
  if (!isfinite(kap.total)) {
    if (isfinite(kap.es)) {
      kap.ff = 0.;
      kap.bf = 0.;
      kap.total = kap.es;
    } else {
      x.err(ERR_NONFINITE, p.number, 1);
    }
  }
}

// ------------------------------------------------------------------------------------------ lines
// rpkt.cc:26-65.  lnu_first, lnu_last: line_nu[0] and line_nu[nlines - 1], loaded once by a caller that walks many
// lines (a dependent load per line otherwise)
DEVFN int closest_transition(int nlines, const double *lnu, double nu_cmf, int next_trans, double lnu_first,
                             double lnu_last) {
  const int left = next_trans;
  const int right = nlines - 1;
  if (nu_cmf < lnu_last) return -1;
  if (left > right) return -1;
  if (left > 0) return left;
  if (nu_cmf >= lnu_first) return 0;
  int lo = next_trans, hi = nlines;
  while (lo < hi) {
    const int mid = lo + (hi - lo) / 2;
    if (!(lnu[mid] <= nu_cmf))
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo;
}
DEVFN int closest_transition(const Ctx &K, double nu_cmf, int next_trans, double lnu_first, double lnu_last) {
  return closest_transition(K.T.nlines, K.T.line_nu, nu_cmf, next_trans, lnu_first, lnu_last);
}
DEVFN int closest_transition(const Ctx &K, double nu_cmf, int next_trans) {
  return closest_transition(K, nu_cmf, next_trans, K.T.line_nu[0], K.T.line_nu[max(K.T.nlines - 1, 0)]);
}
// rpkt.cc:511-555
DEVFN void closest_transition_empty(const Ctx &K, Pkt &p) {
  const int nlines = K.T.nlines;
  const double *lnu = K.T.line_nu;
  const int left = p.next_trans;
  const int right = nlines - 1;
  if (p.nu_cmf < lnu[right]) p.next_trans = nlines + 1;
  if (left > right) p.next_trans = nlines + 1;
  int matchindex;
  if (p.nu_cmf >= lnu[left]) {
    matchindex = left;
  } else {
    int lo = p.next_trans, hi = nlines;
    while (lo < hi) {
      const int mid = lo + (hi - lo) / 2;
      if (!(lnu[mid] <= p.nu_cmf))
        lo = mid + 1;
      else
        hi = mid;
    }
    matchindex = lo;
  }
  p.next_trans = matchindex;
}

// move_pkt_withtime restricted to the fields a dummy packet needs (vectors.h:113-144)
DEVFN void move_dummy(bool rel, double pos[3], const double dir[3], double &t, double &nu_cmf, double nu_rf,
                      double distance) {
  const double nu_cmf_old = nu_cmf;
  t += distance / ARTIS_CLIGHT_PROP;
  pos[0] += (dir[0] * distance);
  pos[1] += (dir[1] * distance);
  pos[2] += (dir[2] * distance);
  nu_cmf = nu_rf * doppler_pos_dir(rel, pos, dir, t);
  if (nu_cmf > nu_cmf_old) nu_cmf = nu_cmf_old;
}
DEVFN void move_dummy(const Ctx &K, double pos[3], const double dir[3], double &t, double &nu_cmf, double nu_rf,
                      double distance) {
  move_dummy((bool)K.R.relativistic_doppler, pos, dir, t, nu_cmf, nu_rf, distance);
}

// The line walk over the per-cell Sobolev coefficient table (DevCells::linecoef): a window of 8 consecutive
// lines' frequencies and coefficients is two 64-byte runs -- four 16-byte loads each, all independent, one trip to
// memory per 8 lines -- staged in the lane's LDS column; no population gathers.  tau_line = coef * dt is the
// reference's (B_lu n_l - B_ul n_u) * HCLIGHTOVERFOURPI * dt evaluated in the same order (k_linecoef).
#define LC_WIN 8
#define WAVE_BLOCK_T 256  // threads per block of the kernels that set Tx::win (k_rpkt: WAVE_BLOCK)
typedef double f64x2 __attribute__((ext_vector_type(2)));
typedef const __attribute__((address_space(1))) f64x2 glb_f64x2;
template <int WIN>
DEVFN void lc_window_n(const double *nu8, const double *coef, __attribute__((address_space(3))) double *win) {
  glb_f64x2 *nu = (glb_f64x2 *)nu8;
  glb_f64x2 *co = (glb_f64x2 *)coef;
  f64x2 a[WIN / 2], b[WIN / 2];
#pragma unroll
  for (int i = 0; i < WIN / 2; i++) {
    a[i] = nu[i];
    b[i] = co[i];
  }
#pragma unroll
  for (int i = 0; i < WIN / 2; i++) {
    win[(2 * i) * WAVE_BLOCK_T] = a[i].x;
    win[(2 * i + 1) * WAVE_BLOCK_T] = a[i].y;
    win[(WIN + 2 * i) * WAVE_BLOCK_T] = b[i].x;
    win[(WIN + 2 * i + 1) * WAVE_BLOCK_T] = b[i].y;
  }
}
DEVFN void lc_window(const double *nu8, const double *coef, __attribute__((address_space(3))) double *win) {
  lc_window_n<LC_WIN>(nu8, coef, win);
}

// One r-packet step (rpkt.cc:623-813) in three parts, so that k_rpkt can spread its line walk over passes:
// rpkt_step_begin (the draw, the boundary, the cases without a walk, get_event's prologue), get_event_walk (the
// walk over the cell's coefficient row, resumable after a bounded number of lines) and rpkt_step_finish (the step's
// end: move, estimators, event or boundary).  do_rpkt_step runs the three back to back.  RStep holds what crosses
// from one part to the next.
struct RStep {
  double sdist, tdist, edist;
  int snext, mgi, oldmgi, k, eventtype;
  bool cross0, find_nextline;
  Kappa kap;
  // get_event's walk (rpkt.cc:112-325): the draw, the distance that ends the search, the comoving frequency there,
  // the continuum opacity; the dummy packet's position, time and frequency, the next line, the staged window
  double tau_rnd, abort_dist, nu_cmf_abort, kap_cont, tau, dist, dpos[3], dt, dnu;
  int dnext, wb;
};
enum { RSTEP_DONE = 0, RSTEP_WALK = 1, RSTEP_END = 2 };

// rpkt.cc:67-110 (get_event's prologue): true when the walk over the cell's coefficient row is set up in S
// (get_event_walk runs it); otherwise the whole search ran here (the population-gather walk) and S.edist /
// S.eventtype hold its result
DEVFN bool get_event_begin(Tx &x, int k, int mgi, Pkt &p, RStep &S, double tau_rnd, double abort_dist) {
  const Ctx &K = x.K;
  Kappa &kap = S.kap;
  int *rpkt_eventtype = &S.eventtype;
  double tau = 0.;
  double dist = 0.;
  double nu_cmf_abort;
  {
    double apos[3] = {p.pos[0], p.pos[1], p.pos[2]};
    double at = p.prop_time, anu = p.nu_cmf;
    move_dummy(K, apos, p.dir, at, anu, p.nu_rf, abort_dist / 2.);
    move_dummy(K, apos, p.dir, at, anu, p.nu_rf, abort_dist / 2.);
    nu_cmf_abort = anu;
  }
  double dpos[3] = {p.pos[0], p.pos[1], p.pos[2]};
  double dt = p.prop_time, dnu = p.nu_cmf;
  int dnext = p.next_trans;
  calculate_kappa_rpkt_cont(x, p, k, mgi, kap);
  STAMP(x, 1);
  const double kap_cont = kap.total * doppler_packet(K, p);
  if (x.win && k < K.C.linecoef_rows) {
    S.tau_rnd = tau_rnd;
    S.abort_dist = abort_dist;
    S.nu_cmf_abort = nu_cmf_abort;
    S.kap_cont = kap_cont;
    S.tau = tau;
    S.dist = dist;
    for (int d = 0; d < 3; d++) S.dpos[d] = dpos[d];
    S.dt = dt;
    S.dnu = dnu;
    S.dnext = dnext;
    S.wb = -16;
    return true;
  }
  const double *pops = K.C.pops + (int64_t)k * K.T.nlevels_total;
  const double lnu_first = K.T.line_nu[0], lnu_last = K.T.line_nu[max(K.T.nlines - 1, 0)];
  unsigned long long nscanned = 0, ntaus = 0;
  double result;
  // The walk visits consecutive lines.  Their 32-byte records and the two level populations each needs (random
  // gathers into the cell's pops) are fetched four lines at a time, all loads independent, so a long walk
  // waits for memory twice per four lines instead of three times per line.
  int pf_base = -16;
  LineTau r0, r1, r2, r3;
  double pl0 = 0, pl1 = 0, pl2 = 0, pl3 = 0, pu0 = 0, pu1 = 0, pu2 = 0, pu3 = 0;
  while (true) {
    const int lineindex = closest_transition(K, dnu, dnext, lnu_first, lnu_last);
    if (lineindex >= 0) {
      nscanned++;
      if ((unsigned)(lineindex - pf_base) >= 4u) {
        pf_base = lineindex;
        const int nl1 = K.T.nlines - 1;
        r0 = K.T.line_tau[lineindex];
        r1 = K.T.line_tau[min(lineindex + 1, nl1)];
        r2 = K.T.line_tau[min(lineindex + 2, nl1)];
        r3 = K.T.line_tau[min(lineindex + 3, nl1)];
        pl0 = pops[r0.ul_lower];
        pu0 = pops[r0.ul_upper];
        pl1 = pops[r1.ul_lower];
        pu1 = pops[r1.ul_upper];
        pl2 = pops[r2.ul_lower];
        pu2 = pops[r2.ul_upper];
        pl3 = pops[r3.ul_lower];
        pu3 = pops[r3.ul_upper];
      }
      const int pj = lineindex - pf_base;
      const double nu_trans = pj == 0 ? r0.nu : pj == 1 ? r1.nu : pj == 2 ? r2.nu : r3.nu;
      dnext = lineindex + 1;
      double ldist;
      if (dnu <= nu_trans) {
        ldist = 0;
      } else if (!K.R.relativistic_doppler) {
        ldist = ARTIS_CLIGHT * dt * (dnu / nu_trans - 1);
      } else {
        const double nu_r = nu_trans / p.nu_rf;
        const double ct = ARTIS_CLIGHT * dt;
        const double r = vec_len(dpos);
        const double mu = dot(p.dir, dpos) / r;
        ldist = -mu * r + (ct - nu_r * nu_r * sqrt(ct * ct - (1 + r * r * (1 - mu * mu) * (1 + pow(nu_r, -2))))) /
                              (1 + nu_r * nu_r);
      }
      if (ldist < 0.) {
        if (!(ldist >= -100.)) {
          x.err(ERR_LDIST, p.number, lineindex);
          result = 0.;
          break;
        }
        ldist = 0.;
      }
      const double tau_cont = kap_cont * ldist;
      if (tau_rnd - tau > tau_cont) {
        if (nu_trans < nu_cmf_abort) {
          dnext -= 1;
          p.next_trans = dnext;
          result = DBL_MAX;
          break;
        }
        const double n_u = pj == 0 ? pu0 : pj == 1 ? pu1 : pj == 2 ? pu2 : pu3;
        const double n_l = pj == 0 ? pl0 : pj == 1 ? pl1 : pj == 2 ? pl2 : pl3;
        const double B_lu = pj == 0 ? r0.B_lu : pj == 1 ? r1.B_lu : pj == 2 ? r2.B_lu : r3.B_lu;
        const double B_ul = pj == 0 ? r0.B_ul : pj == 1 ? r1.B_ul : pj == 2 ? r2.B_ul : r3.B_ul;
        double tau_line = (B_lu * n_l - B_ul * n_u) * ARTIS_HCLIGHTOVERFOURPI * dt;
        ntaus++;
        if (tau_line < 0) tau_line = 0.;
        if (tau_rnd - tau > tau_cont + tau_line) {
          dist = dist + ldist;
          tau += tau_cont + tau_line;
          move_dummy(K, dpos, p.dir, dt, dnu, p.nu_rf, ldist);
        } else {
          p.ma_element = K.T.line_elem[lineindex];
          p.ma_ion = K.T.line_ion[lineindex];
          p.ma_level = K.T.line_upper[lineindex];
          p.ma_activatingline = lineindex;
          double edist = dist + ldist;
          if (edist >= abort_dist) edist = abort_dist * (1 - 2e-8);
          *rpkt_eventtype = ARTIS_RPKT_EVENTTYPE_BB;
          p.next_trans = dnext;
          result = edist;
          break;
        }
      } else {
        const double edist = dist + (tau_rnd - tau) / kap_cont;
        dnext -= 1;
        *rpkt_eventtype = ARTIS_RPKT_EVENTTYPE_CONT;
        p.next_trans = dnext;
        result = edist;
        break;
      }
    } else {
      dnext = K.T.nlines + 1;
      const double tau_cont = kap_cont * (abort_dist - dist);
      double edist;
      if (tau_rnd - tau > tau_cont) {
        edist = DBL_MAX;
      } else {
        edist = dist + (tau_rnd - tau) / kap_cont;
        *rpkt_eventtype = ARTIS_RPKT_EVENTTYPE_CONT;
      }
      p.next_trans = dnext;
      result = edist;
      break;
    }
  }
  lwork(x.L, WK_LINES_SCANNED, nscanned);
  lwork(x.L, WK_LINE_TAUS, ntaus);
  x.wl += (unsigned)nscanned;
  STAMP(x, 2);
  S.edist = result;
  return false;
}


// rpkt.cc:112-325 over the cell's coefficient row (DevCells::linecoef) in 8-line LDS windows: at most `budget`
// lines per call; false when the budget ran out first (S holds the walk, the next call continues it), true when the
// search ended (S.edist, S.eventtype; p.next_trans and, for a line event, the macro-atom activation fields set)
DEVFN bool get_event_walk(Tx &x, Pkt &p, RStep &S, int budget) {
  const Ctx &K = x.K;
  int *rpkt_eventtype = &S.eventtype;
  const double tau_rnd = S.tau_rnd, abort_dist = S.abort_dist, nu_cmf_abort = S.nu_cmf_abort, kap_cont = S.kap_cont;
  double tau = S.tau, dist = S.dist;
  double dpos[3] = {S.dpos[0], S.dpos[1], S.dpos[2]};
  double dt = S.dt, dnu = S.dnu;
  int dnext = S.dnext;
  const double lnu_first = K.T.line_nu[0], lnu_last = K.T.line_nu[max(K.T.nlines - 1, 0)];
  unsigned long long nscanned = 0, ntaus = 0;
  double result = 0.;
  bool done = true;
  // the context fields the walk reads, in registers: through the context pointer they are reloaded from memory
  // on every line (the compiler cannot prove the kernel's stores leave them unchanged)
  __attribute__((address_space(3))) double *win = x.win;
  const bool rel = K.R.relativistic_doppler;
  const int nlines = K.T.nlines;
  const double *lnu = K.T.line_nu, *nu8 = K.T.line_nu8;
  const double *crow = K.C.linecoef + (int64_t)S.k * K.C.linecoef_stride;
  int wb = S.wb;
  while (true) {
    if (budget-- == 0) {  // resume next call
      done = false;
      S.tau = tau;
      S.dist = dist;
      for (int d = 0; d < 3; d++) S.dpos[d] = dpos[d];
      S.dt = dt;
      S.dnu = dnu;
      S.dnext = dnext;
      S.wb = wb;
      break;
    }
    const int lineindex = closest_transition(nlines, lnu, dnu, dnext, lnu_first, lnu_last);
    if (lineindex >= 0) {
      nscanned++;
      if ((unsigned)(lineindex - wb) >= (unsigned)LC_WIN) {
        wb = lineindex & ~(LC_WIN - 1);
        lc_window(nu8 + wb, crow + wb, win);
      }
      const int pj = lineindex - wb;
      const double nu_trans = win[pj * WAVE_BLOCK_T];
      dnext = lineindex + 1;
      double ldist;
      if (dnu <= nu_trans) {
        ldist = 0;
      } else if (!rel) {
        ldist = ARTIS_CLIGHT * dt * (dnu / nu_trans - 1);
      } else {
        const double nu_r = nu_trans / p.nu_rf;
        const double ct = ARTIS_CLIGHT * dt;
        const double r = vec_len(dpos);
        const double mu = dot(p.dir, dpos) / r;
        ldist = -mu * r + (ct - nu_r * nu_r * sqrt(ct * ct - (1 + r * r * (1 - mu * mu) * (1 + pow(nu_r, -2))))) /
                              (1 + nu_r * nu_r);
      }
      if (ldist < 0.) {
        if (!(ldist >= -100.)) {
          x.err(ERR_LDIST, p.number, lineindex);
          result = 0.;
          break;
        }
        ldist = 0.;
      }
      const double tau_cont = kap_cont * ldist;
      if (tau_rnd - tau > tau_cont) {
        if (nu_trans < nu_cmf_abort) {
          dnext -= 1;
          p.next_trans = dnext;
          result = DBL_MAX;
          break;
        }
        double tau_line = win[(LC_WIN + pj) * WAVE_BLOCK_T] * dt;
        ntaus++;
        if (tau_line < 0) tau_line = 0.;
        if (tau_rnd - tau > tau_cont + tau_line) {
          dist = dist + ldist;
          tau += tau_cont + tau_line;
          move_dummy(rel, dpos, p.dir, dt, dnu, p.nu_rf, ldist);
        } else {
          p.ma_element = K.T.line_elem[lineindex];
          p.ma_ion = K.T.line_ion[lineindex];
          p.ma_level = K.T.line_upper[lineindex];
          p.ma_activatingline = lineindex;
          double edist = dist + ldist;
          if (edist >= abort_dist) edist = abort_dist * (1 - 2e-8);
          *rpkt_eventtype = ARTIS_RPKT_EVENTTYPE_BB;
          p.next_trans = dnext;
          result = edist;
          break;
        }
      } else {
        const double edist = dist + (tau_rnd - tau) / kap_cont;
        dnext -= 1;
        *rpkt_eventtype = ARTIS_RPKT_EVENTTYPE_CONT;
        p.next_trans = dnext;
        result = edist;
        break;
      }
    } else {
      dnext = K.T.nlines + 1;
      const double tau_cont = kap_cont * (abort_dist - dist);
      double edist;
      if (tau_rnd - tau > tau_cont) {
        edist = DBL_MAX;
      } else {
        edist = dist + (tau_rnd - tau) / kap_cont;
        *rpkt_eventtype = ARTIS_RPKT_EVENTTYPE_CONT;
      }
      p.next_trans = dnext;
      result = edist;
      break;
    }
  }
  lwork(x.L, WK_LINES_SCANNED, nscanned);
  lwork(x.L, WK_LINE_TAUS, ntaus);
  x.wl += (unsigned)nscanned;
  STAMP(x, 2);
  if (done) S.edist = result;
  return done;
}

// rpkt.cc:557-621 + radfield.cc:831-876
DEVFN void update_estimators(Tx &x, const Pkt &p, const Kappa &kap, double distance) {
  const Ctx &K = x.K;
  const int mgi = cell_mgi(K, p.where);
  if (mgi == K.G.npts_model) return;
  const int k = K.C.ne_index[mgi];
  lwork(x.L, WK_EST_SEGMENTS, 1);
  const double distance_e_cmf = distance * p.e_cmf;
  const double nu = p.nu_cmf;
  const int nne = K.C.n_nonempty;
  if (x.est_lds && K.C.est_lds_J >= 0) {
    double *e = x.est_lds + K.C.est_lds_J;
    atomicAdd(&e[k], distance_e_cmf);
    atomicAdd(&e[nne + k], distance_e_cmf * nu);
    atomicAdd(&e[2 * nne + k], distance_e_cmf * kap.ffheating);
  } else if (x.defer_est) {
    x.est_mgi = mgi;
    x.est_de = distance_e_cmf;
    x.est_denu = distance_e_cmf * nu;
    x.est_deff = distance_e_cmf * kap.ffheating;
  } else {
    safeadd(&K.E.J[mgi], distance_e_cmf);
    safeadd(&K.E.nuJ[mgi], distance_e_cmf * nu);
    safeadd(&K.E.ffheat[mgi], distance_e_cmf * kap.ffheating);
  }
  if (K.R.detailed_bf && distance_e_cmf != 0) {
    // radfield.cc:764-829 update_bfestimators: gamma_contr[i] at the frequency the opacity was computed at
    // (rpkt.cc:1166-1171; zero for continua above kap.nu or not included), the window test at the current nu
    const double dopplerfactor = doppler_packet(K, p);
    const double d_over_nu = distance_e_cmf / nu * dopplerfactor;
    const int64_t row = (int64_t)mgi * K.T.nbf;
    if (x.defer_bf) {  // (k_rpkt: added by the wave after the step, wave_bf_estimators)
      x.bf_pend = K.R.do_r_lc != 0;
      x.bf_k = k;
      x.bf_mgi = mgi;
      x.bf_nu = nu;
      x.bf_kapnu = kap.nu;
      x.bf_d = d_over_nu;
    } else {
      // the window nu_edge <= nu <= nu_max of the reference's loop is [lo, hi) (bf_range); gamma_contr is zero
      // below the first continuum kap.nu reaches (lo_k), and adding zero changes no sum, so the loop starts at
      // max(lo, lo_k) (without do_r_lc no bf opacity is evaluated and the zero-initialised gamma_contr stays 0,
      // rpkt.cc:1230)
      int lo, hi, lo_k, hi_k;
      bf_range(K, nu, lo, hi);
      bf_range(K, kap.nu, lo_k, hi_k);
      const BfCell cell = bf_cell(K, k, mgi, kap.nu);
      for (int i = max(lo, lo_k); K.R.do_r_lc && i < hi; i++) {
        double gc = 0., nnlevel;
        if (kap.nu < K.T.allcont_nu_edge[i] || !bf_contribution(K, cell, i, kap.nu, &nnlevel, &gc)) continue;
        if (x.est_lds && K.C.est_lds_bf >= 0)
          atomicAdd(&x.est_lds[K.C.est_lds_bf + (int64_t)k * K.T.nbf + i], gc * d_over_nu);
        else
          safeadd(&K.E.bfrate[row + i], gc * d_over_nu);
      }
    }
  }
  if (K.R.multibin) {  // radfield.cc:845-866
    const int b = rf_select_bin(K, nu);
    if (b >= 0 && x.est_lds && K.C.est_lds_rf >= 0) {
      double *e = x.est_lds + K.C.est_lds_rf + 3 * ((int64_t)k * K.T.rf_nbins + b);
      atomicAdd(&e[0], distance_e_cmf);
      atomicAdd(&e[1], distance_e_cmf * nu);
      atomicAdd(&e[2], 1.);
    } else if (b >= 0) {
      const int64_t mb = (int64_t)mgi * K.T.rf_nbins + b;
      safeadd(&K.E.rfJ[mb], distance_e_cmf);
      safeadd(&K.E.rfnuJ[mb], distance_e_cmf * nu);
      safeadd(&K.E.rfcount[mb], 1.);
    }
  }
  // the ground-continuum estimators exist unless both NO_LUT_PHOTOION and NO_LUT_BFHEATING (rpkt.cc:573-614)
  if (K.R.no_lut_photoion && K.R.no_lut_bfheating) return;
  const double distance_e_cmf_over_nu = distance_e_cmf / nu;
  const BfCell cell = bf_cell(K, k, mgi, kap.nu);
  for (int g = 0; g < K.T.nbfg; g++) {
    const double nu_edge = K.T.groundcont_nu_edge[g];
    if (nu > nu_edge) {
      const int element = K.T.groundcont_element[g];
      if (K.C.elem_abundance[(int64_t)mgi * K.T.nelements + element] > 0) {
        // groundcont_gamma_contr[g] at the frequency the opacity was computed at (rpkt.cc:1166-1171)
        // (zero without do_r_lc: calculate_kappa_bf_gammacontr never runs, input.cc:1462-1468, rpkt.cc:1230)
        double gcontr = 0.;
        for (int q = K.T.gc_cont_off[g]; K.R.do_r_lc && q < K.T.gc_cont_off[g + 1]; q++) {  // ascending allcont order
          const int i = K.T.gc_cont[q];
          if (kap.nu < K.T.allcont_nu_edge[i]) break;
          double nnlevel, gc;
          if (bf_contribution(K, cell, i, kap.nu, &nnlevel, &gc)) gcontr += gc;
        }
        const int ion = K.T.groundcont_ion[g];
        const int64_t idx = (int64_t)mgi * K.T.nelements * K.T.maxnions + element * K.T.maxnions + ion;
        if (!K.R.no_lut_photoion) safeadd(&K.E.gamma[idx], gcontr * distance_e_cmf_over_nu);
        if (!K.R.no_lut_bfheating) safeadd(&K.E.bfheat[idx], gcontr * distance_e_cmf * (1. - nu_edge / nu));
        lwork(x.L, WK_GC_UPDATES, 1);
      }
    } else {
      break;
    }
  }
}

// The deferred J / nuJ / ffheating terms of a converged wave (radfield.cc:831-836, rpkt.cc:569-579; N1): when all
// the wave's contributing lanes are in one cell -- the common case of few-cell models, where per-lane atomics on
// the same three addresses serialise -- the terms are summed across the wave and added by one lane; otherwise
// every lane adds its own.  Float atomics are unordered either way, so the sums agree to rounding.
DEVFN void wave_flush_estimators(Tx &x) {
  const Ctx &K = x.K;
  const bool pend = x.est_mgi >= 0;
  const unsigned long long pm = __ballot(pend);
  if (pm) {
    const int leader = __ffsll((long long)pm) - 1;
    const int m0 = __shfl(x.est_mgi, leader, 64);
    if (__ballot(pend && x.est_mgi != m0) == 0) {
      double a = pend ? x.est_de : 0., b = pend ? x.est_denu : 0., c = pend ? x.est_deff : 0.;
      for (int off = 32; off > 0; off >>= 1) {
        a += __shfl_xor(a, off, 64);
        b += __shfl_xor(b, off, 64);
        c += __shfl_xor(c, off, 64);
      }
      if ((int)__lane_id() == leader) {
        safeadd(&K.E.J[m0], a);
        safeadd(&K.E.nuJ[m0], b);
        safeadd(&K.E.ffheat[m0], c);
      }
    } else if (pend) {
      safeadd(&K.E.J[x.est_mgi], x.est_de);
      safeadd(&K.E.nuJ[x.est_mgi], x.est_denu);
      safeadd(&K.E.ffheat[x.est_mgi], x.est_deff);
    }
  }
  x.est_mgi = -1;
}

DEVFN double readlane_d(double v, int l) {
  const uint64_t u = (uint64_t)__double_as_longlong(v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), l);
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
// ---- the continuum sums of a step made by the whole wave (k_rpkt, models with many bf continua per frequency) ----
// Every lane contributes n consecutive items (its continua); the wave's items are laid out lane after lane
// (exclusive prefix `pref` over the lanes), and each pass over them gives every lane one item -- so a wave spends
// about total / 64 item evaluations instead of the longest lane's count.  Wave-uniform.
DEVFN int wave_excl_prefix(int n, int &total) {
  const int lane = (int)__lane_id();
  int incl = n;
  for (int off = 1; off < 64; off <<= 1) {
    const int t = __shfl_up(incl, off, 64);
    if (lane >= off) incl += t;
  }
  total = __shfl(incl, 63, 64);
  return incl - n;
}
// the lane owning item j: the last lane whose prefix is <= j (lane prefixes in the wave's LDS slots s_pref[0..63])
DEVFN int wave_item_owner(const int *s_pref, int j) {
  int o = 0;
#pragma unroll
  for (int step = 32; step > 0; step >>= 1)
    if (s_pref[o + step] <= j) o += step;
  return o;
}
DEVFN const double2 *shfl_ptr(const double2 *p, int src) {
  return (const double2 *)__shfl((long long)p, src, 64);
}
// The wave's item loops take COOP_UNR items per lane per trip (bf_contribution_batch: their table loads in flight
// together); the LDS slots coop_d hold 64 * COOP_UNR terms per wave.
#define COOP_UNR 4
// calculate_kappa_bf_gammacontr's kappa_bf sum (rpkt.cc:1075-1207) of every lane with `want` (cell k / mgi,
// frequency nu): the terms n_level * gamma_contr are evaluated by the wave 64 * COOP_UNR at a time into the LDS slots
// s_d, and each lane adds its own terms in continuum order -- the reference's sum, term for term.  *hi: the continua
// the reference's loop visits (the work counter).
DEVFN double wave_kappa_bf(Tx &x, bool want, int k, int mgi, double nu, int &hi_out) {
  const Ctx &K = x.K;
  double *s_d = x.coop_d;
  int *s_i = x.coop_i;
  const int lane = (int)__lane_id();
  int lo = 0, hi = 0;
  if (want) bf_range(K, nu, lo, hi);
  hi_out = hi;
  const int n = hi - lo;
  int total;
  const int pref = wave_excl_prefix(n, total);
  double sum = 0.;
  if (total == 0) return sum;
  const BfCell cell = want ? bf_cell(K, k, mgi, nu) : BfCell{K.C.bfcell, 0.};
  s_i[lane] = pref;
  __builtin_amdgcn_wave_barrier();
  constexpr int U = COOP_UNR;
  for (int c0 = 0; c0 < total; c0 += 64 * U) {
    BfCell cl[U];
    int ci[U];
    double nuu[U], nn[U], gc[U];
    bool ok[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int j = min(c0 + u * 64 + lane, total - 1);
      const int o = wave_item_owner(s_i, j);
      ci[u] = __shfl(lo, o, 64) + (j - __shfl(pref, o, 64));
      nuu[u] = __shfl(nu, o, 64);
      cl[u] = BfCell{shfl_ptr(cell.row, o), __shfl(cell.expfac, o, 64)};
    }
    bf_contribution_batch<U>(K, cl, ci, nuu, ok, nn, gc);
#pragma unroll
    for (int u = 0; u < U; u++) s_d[u * 64 + lane] = (c0 + u * 64 + lane < total && ok[u]) ? nn[u] * gc[u] : 0.;
    __builtin_amdgcn_wave_barrier();
    const int a = max(pref, c0), b = min(pref + n, c0 + 64 * U);
    for (int jj = a; jj < b; jj++) sum += s_d[jj - c0];
    __builtin_amdgcn_wave_barrier();
  }
  return sum;
}
// update_bfestimators (radfield.cc:764-829) of the step, deferred by update_estimators (Tx::defer_bf): the window
// [max(lo(nu), lo(kap.nu)), hi(nu)) of every pending lane, gamma_contr at kap.nu, made by the wave 64 * COOP_UNR
// continua at a time; each term is added to the estimator on its own (the additions are atomics, in no order, as
// per lane).
DEVFN void wave_bf_estimators(Tx &x) {
  const Ctx &K = x.K;
  const int lane = (int)__lane_id();
  const bool want = x.bf_pend;
  x.bf_pend = false;
  int start = 0, n = 0;
  if (want) {
    int lo, hi, lo_k, hi_k;
    bf_range(K, x.bf_nu, lo, hi);
    bf_range(K, x.bf_kapnu, lo_k, hi_k);
    start = max(lo, lo_k);
    n = max(0, hi - start);
  }
  int total;
  const int pref = wave_excl_prefix(n, total);
  if (total == 0) return;
  const BfCell cell = want ? bf_cell(K, x.bf_k, x.bf_mgi, x.bf_kapnu) : BfCell{K.C.bfcell, 0.};
  x.coop_i[lane] = pref;
  __builtin_amdgcn_wave_barrier();
  const int nbf = K.T.nbf;
  const bool lds = x.est_lds && K.C.est_lds_bf >= 0;
  constexpr int U = COOP_UNR;
  for (int c0 = 0; c0 < total; c0 += 64 * U) {
    BfCell cl[U];
    int ci[U], ko[U], mo[U];
    double nuu[U], nn[U], gc[U], dd[U];
    bool ok[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int j = min(c0 + u * 64 + lane, total - 1);
      const int o = wave_item_owner(x.coop_i, j);
      ci[u] = __shfl(start, o, 64) + (j - __shfl(pref, o, 64));
      ko[u] = __shfl(x.bf_k, o, 64);
      mo[u] = __shfl(x.bf_mgi, o, 64);
      nuu[u] = __shfl(x.bf_kapnu, o, 64);
      dd[u] = __shfl(x.bf_d, o, 64);
      cl[u] = BfCell{shfl_ptr(cell.row, o), __shfl(cell.expfac, o, 64)};
    }
    bf_contribution_batch<U>(K, cl, ci, nuu, ok, nn, gc);
#pragma unroll
    for (int u = 0; u < U; u++) {
      // (the window's lower edges: the continua below kap.nu's, nu <= nu_edge excluded as update_bfestimators does)
      if (c0 + u * 64 + lane < total && ok[u] && !(nuu[u] < K.T.allcont_nu_edge[ci[u]])) {
        if (lds)
          atomicAdd(&x.est_lds[K.C.est_lds_bf + (int64_t)ko[u] * nbf + ci[u]], gc[u] * dd[u]);
        else
          safeadd(&K.E.bfrate[(int64_t)mo[u] * nbf + ci[u]], gc[u] * dd[u]);
      }
    }
  }
  __builtin_amdgcn_wave_barrier();
}
// rpkt.cc:370-447, the continuum selection of a bound-free absorption (rpkt_event_continuum, deferred with
// Tx::defer_sel), then the rest of that event.  For each pending lane in turn the wave evaluates the terms
// n_level * gamma_contr 64 * COOP_UNR at a time into LDS, and every lane runs the reference's running sum over them
// in order (the first continuum at which it reaches the draw; the last one if none): the reference's linear search,
// term for term.  Wave-uniform.
DEVFN void wave_bf_select(Tx &x, Pkt &p, uint64_t *__restrict__ soa, int64_t n, int64_t idx) {
  const Ctx &K = x.K;
  unsigned long long m = __ballot(x.sel_pend);
  if (!m) return;
  const int lane = (int)__lane_id();
  const int last = K.T.nbf - 1;
  constexpr int U = COOP_UNR;
  int sel = last;
  for (; m; m &= m - 1) {
    const int o = __ffsll((long long)m) - 1;
    const int k = __builtin_amdgcn_readlane(x.sel_k, o), mgi = __builtin_amdgcn_readlane(x.sel_mgi, o);
    const double nu = readlane_d(x.sel_nu, o), rnd = readlane_d(x.sel_rand, o);
    int found = last;
    double running = 0.;
    if (!(running < rnd)) {
      found = 0;
    } else {
      int lo, hi;
      bf_range(K, nu, lo, hi);
      const int end = min(hi, last);
      const BfCell cell = bf_cell(K, k, mgi, nu);
      bool done = false;
      for (int c0 = lo; c0 < end && !done; c0 += 64 * U) {
        BfCell cl[U];
        int ci[U];
        double nuu[U], nn[U], gc[U];
        bool ok[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
          ci[u] = min(c0 + u * 64 + lane, end - 1);
          nuu[u] = nu;
          cl[u] = cell;
        }
        bf_contribution_batch<U>(K, cl, ci, nuu, ok, nn, gc);
#pragma unroll
        for (int u = 0; u < U; u++) x.coop_d[u * 64 + lane] = (c0 + u * 64 + lane < end && ok[u]) ? nn[u] * gc[u] : 0.;
        __builtin_amdgcn_wave_barrier();
        const int cend = min(end, c0 + 64 * U);
        for (int i = c0; i < cend; i++) {
          running += x.coop_d[i - c0];
          if (!(running < rnd)) {
            found = i;
            done = true;
            break;
          }
        }
        __builtin_amdgcn_wave_barrier();
      }
    }
    if (lane == o) sel = found;
  }
  if (x.sel_pend) {
    x.sel_pend = false;
    const int element = K.T.allcont_element[sel];
    const int ion = K.T.allcont_ion[sel];
    const double zrand3 = artis_rng_uniform(&x.rng);
    if (zrand3 < K.T.allcont_nu_edge[sel] / p.nu_cmf) {
      lctr(x.L, CTR_MA_STAT_ACTIVATION_BF);
      p.interactions += 1;
      p.last_event = 3;
      p.type = ARTIS_TYPE_MA;
      p.ma_element = element;
      p.ma_ion = ion + 1;
      p.ma_level = get_phixsupperlevel(K, element, ion, K.T.allcont_level[sel], K.T.allcont_target[sel]);
      p.ma_activatingline = -99;
      soa[PW(n, idx, 36)] = pack2(p.ma_element, p.ma_ion);  // (the record's macro-atom state, cold words)
      soa[PW(n, idx, 37)] = pack2(p.ma_level, p.ma_activatingline);
    } else {
      lctr(x.L, CTR_K_STAT_FROM_BF);
      p.interactions += 1;
      p.last_event = 4;
      p.type = ARTIS_TYPE_KPKT;
    }
  }
}

// the block's LDS estimator accumulator: zeroed at the start of k_rpkt, added to the estimators at its end (one
// atomic per non-zero entry and block)
__host__ __device__ inline bool est_lds_on(const Ctx &K) { return K.C.est_lds_J >= 0 || K.C.est_lds_bf >= 0 || K.C.est_lds_rf >= 0; }
DEVFN void est_lds_zero(double *e) {
  for (int i = threadIdx.x; i < EST_LDS_DOUBLES; i += blockDim.x) e[i] = 0.;
  __syncthreads();
}
DEVFN void est_lds_flush(const Ctx &K, const double *e) {
  __syncthreads();
  const int nne = K.C.n_nonempty;
  if (K.C.est_lds_J >= 0)
    for (int i = threadIdx.x; i < 3 * nne; i += blockDim.x) {
      const double v = e[K.C.est_lds_J + i];
      if (v == 0.) continue;
      const int mgi = K.C.ne_mgi[i % nne];
      safeadd(i < nne ? &K.E.J[mgi] : i < 2 * nne ? &K.E.nuJ[mgi] : &K.E.ffheat[mgi], v);
    }
  if (K.C.est_lds_bf >= 0) {
    const int nbf = K.T.nbf;
    for (int i = threadIdx.x; i < nne * nbf; i += blockDim.x) {
      const double v = e[K.C.est_lds_bf + i];
      if (v != 0.) safeadd(&K.E.bfrate[(int64_t)K.C.ne_mgi[i / nbf] * nbf + i % nbf], v);
    }
  }
  if (K.C.est_lds_rf >= 0) {
    const int nb = K.T.rf_nbins;
    for (int i = threadIdx.x; i < 3 * nne * nb; i += blockDim.x) {
      const double v = e[K.C.est_lds_rf + i];
      if (v == 0.) continue;
      const int cb = i / 3;
      const int64_t mb = (int64_t)K.C.ne_mgi[cb / nb] * nb + cb % nb;
      safeadd((i % 3) == 0 ? &K.E.rfJ[mb] : (i % 3) == 1 ? &K.E.rfnuJ[mb] : &K.E.rfcount[mb], v);
    }
  }
}

// ------------------------------------------------------------------------------------------ virtual packets
// vpkt.cc:837-896, the part at the emission site: the cut on thick cells and the observer time / frequency
// windows.  A packet passing some window is recorded in the spawn buffer; the traversals themselves run in
// k_vpkt (vpkt.h), which repeats the per-observer cuts.  The next_trans fix-up of vpkt.cc:853-858 only ever
// writes 0 over 0 and is omitted.
// one slot of counter *c per active lane, one atomic per wave (made by the first active lane)
DEVFN uint32_t wave_slot(uint32_t *c) {
  const unsigned long long mask = __ballot(1);
  const int leader = __ffsll((long long)mask) - 1;
  uint32_t base = 0;
  if ((int)__lane_id() == leader) base = atomicAdd(c, (uint32_t)__popcll(mask));
  base = __shfl(base, leader, 64);
  return base + (uint32_t)__popcll(mask & ((1ull << __lane_id()) - 1ull));
}

DEVFN void vpkt_spawn(Tx &x, const Pkt &p, int realtype) {
  const Ctx &K = x.K;
  const DevVpkt &V = K.V;
  const int mgi = cell_mgi(K, p.where);
  if (mgi == K.G.npts_model || K.C.thick[mgi] != 0) return;
  const double t_current = p.prop_time;
  bool any = false;
  for (int b = 0; b < V.nobs && !any; b++) {
    const double obs[3] = {V.obs[3 * b], V.obs[3 * b + 1], V.obs[3 * b + 2]};
    const double t_arrive = t_current - (dot(p.pos, obs) / ARTIS_CLIGHT_PROP);
    if (t_arrive >= V.tmin_input && t_arrive <= V.tmax_input) {
      const double nu_rf = p.nu_cmf / doppler_pos_dir(K, p.pos, obs, t_current);
      for (int i = 0; i < V.nrange; i++)
        if (nu_rf > V.numin_input[i] && nu_rf < V.numax_input[i]) any = true;
    }
  }
  if (!any) return;
  uint32_t s = wave_slot(&V.spawn_ctr[0]);  // (the buffer order is free: k_vpkt sorts or traces it in any order)
  int64_t cap = V.cap;
  double *sp = V.spawn;
  if (s >= V.cap) {  // full: an overflow record, and the packet is parked by its kernel
    *(volatile uint32_t *)V.full = 1u;
    x.vstop = true;
    s = atomicAdd(V.ovf_ctr, 1u);
    if (s >= V.ovf_cap) {
      fail(K, ERR_VPKT_OVERFLOW, p.number, (int)V.ovf_cap);
      x.ok = false;
      return;
    }
    cap = V.ovf_cap;
    sp = V.ovf;
  }
  for (int d = 0; d < 3; d++) {
    sp[d * cap + s] = p.pos[d];
    sp[(3 + d) * cap + s] = p.dir[d];
  }
  sp[6 * cap + s] = p.nu_cmf;
  sp[7 * cap + s] = p.e_cmf;
  sp[8 * cap + s] = p.stokes[1];
  sp[9 * cap + s] = p.stokes[2];
  sp[10 * cap + s] = t_current;
  reinterpret_cast<uint64_t *>(sp)[11 * cap + s] = pack2(p.where, p.next_trans);
  reinterpret_cast<uint64_t *>(sp)[12 * cap + s] = pack2(p.last_cross, realtype);
}

// rpkt.cc:330-447
DEVNI void rpkt_event_continuum(Tx &x, Pkt &p, const Kappa &kap, int k, int mgi) {
  const Ctx &K = x.K;
  const double nu = p.nu_cmf;
  const double dopplerfactor = doppler_packet(K, p);
  const double kappa_cont = kap.total * dopplerfactor;
  const double sigma = kap.es * dopplerfactor;
  const double kappa_ff = kap.ff * dopplerfactor;
  const double kappa_bf = kap.bf * dopplerfactor;
  const double zrand = artis_rng_uniform(&x.rng);
  lwork(x.L, WK_CONT_EVENTS, 1);
  if (zrand * kappa_cont < sigma) {
    p.interactions += 1;
    p.nscatterings += 1;
    p.last_event = 12;
    lctr(x.L, CTR_ESCOUNTER);
    lwork(x.L, WK_ES_SCAT, 1);
    if (K.V.on) {  // rpkt.cc:358-363
      p.last_cross = ARTIS_NONE;
      vpkt_spawn(x, p, 1);
    }
    escat_rpkt(x, p);
    p.em_pos[0] = p.pos[0];
    p.em_pos[1] = p.pos[1];
    p.em_pos[2] = p.pos[2];
    p.em_time = (int)p.prop_time;
  } else if (zrand * kappa_cont < sigma + kappa_ff) {
    lctr(x.L, CTR_K_STAT_FROM_FF);
    p.interactions += 1;
    p.last_event = 5;
    p.type = ARTIS_TYPE_KPKT;
    p.absorptiontype = -1;
  } else if (zrand * kappa_cont < sigma + kappa_ff + kappa_bf) {
    p.absorptiontype = -2;
    const double kappa_bf_inrest = kap.bf;
    const double zrand2 = artis_rng_uniform(&x.rng);
    const double kappa_bf_rand = zrand2 * kappa_bf_inrest;
    if (x.defer_sel) {  // (k_rpkt, detailed-bf models: the selection and the rest of the event by the wave)
      x.sel_pend = true;
      x.sel_k = k;
      x.sel_mgi = mgi;
      x.sel_nu = kap.nu;
      x.sel_rand = kappa_bf_rand;
      return;
    }
    // lower_bound over kappa_bf_sum[0, nbf-1): re-scan the running sum of calculate_kappa_bf_gammacontr at the
    // frequency the opacity was computed at
    const int last = K.T.nbf - 1;
    int allcontindex = last;
    double running = 0.;
    const BfCell cell = bf_cell(K, k, mgi, kap.nu);
    // the terms are zero outside [lo, hi) (bf_range): below lo the running sum stays 0 (so the search ends at i = 0
    // only for a zero draw), from hi on it stays at its total (the search then runs on to `last`)
    int lo, hi;
    bf_range(K, kap.nu, lo, hi);
    if (!(running < kappa_bf_rand)) {
      allcontindex = 0;
    } else {
      for (int i = lo; i < min(hi, last); i++) {
        double nnlevel, gc;
        if (bf_contribution(K, cell, i, kap.nu, &nnlevel, &gc)) running += nnlevel * gc;
        if (!(running < kappa_bf_rand)) {
          allcontindex = i;
          break;
        }
      }
    }
    const double nu_edge = K.T.allcont_nu_edge[allcontindex];
    const int element = K.T.allcont_element[allcontindex];
    const int ion = K.T.allcont_ion[allcontindex];
    const int level = K.T.allcont_level[allcontindex];
    const int phixstargetindex = K.T.allcont_target[allcontindex];
    const double zrand3 = artis_rng_uniform(&x.rng);
    if (zrand3 < nu_edge / nu) {
      lctr(x.L, CTR_MA_STAT_ACTIVATION_BF);
      p.interactions += 1;
      p.last_event = 3;
      p.type = ARTIS_TYPE_MA;
      p.ma_element = element;
      p.ma_ion = ion + 1;
      p.ma_level = get_phixsupperlevel(K, element, ion, level, phixstargetindex);
      p.ma_activatingline = -99;
    } else {
      lctr(x.L, CTR_K_STAT_FROM_BF);
      p.interactions += 1;
      p.last_event = 4;
      p.type = ARTIS_TYPE_KPKT;
    }
  } else {
    x.err(ERR_CONT, p.number, 0);
  }
}
// rpkt.cc:449-489
DEVFN void rpkt_event_boundbound(Tx &x, Pkt &p) {
  lctr(x.L, CTR_MA_STAT_ACTIVATION_BB);
  lwork(x.L, WK_BB_EVENTS, 1);
  p.interactions += 1;
  p.last_event = 1;
  p.absorptiontype = p.ma_activatingline;
  p.absorptionfreq = p.nu_rf;
  p.absorptiondir[0] = p.dir[0];
  p.absorptiondir[1] = p.dir[1];
  p.absorptiondir[2] = p.dir[2];
  p.type = ARTIS_TYPE_MA;
  if (x.K.R.record_linestat) atomicAdd(&x.K.E.acounter[p.next_trans - 1], 1);
}

// rpkt.cc:491-509: grey thick cell, coherent electron scattering into a new direction
DEVNI void rpkt_event_thickcell(Tx &x, Pkt &p) {
  p.interactions += 1;
  p.nscatterings += 1;
  p.last_event = 12;
  lctr(x.L, CTR_ESCOUNTER);
  emitt_rpkt(x, p);
  for (int d = 0; d < 3; d++) p.em_pos[d] = p.pos[d];
  p.em_time = (int)p.prop_time;
}

// grey_emissivities.cc:79-122 rlc_emiss_rpkt (do_rlc_est 1 or 2, rpkt.cc:739-741, 769-771, 791-793): the grey
// destruction rate of r-packets, at the segment midpoint; kappagrey * rho is a float product as in the reference.
// An empty cell would add rho = 0 to the reference's extra slot rpkt_emiss[npts_model]: skipped.
DEVFN void rlc_emiss_rpkt(const Ctx &K, const Pkt &p, double dist) {
  const int mgi = cell_mgi(K, p.where);
  if (mgi == K.G.npts_model) return;
  if (dist > 0.0) {
    const double t = p.prop_time;
    const double vel_vec[3] = {p.pos[0] / t, p.pos[1] / t, p.pos[2] / t};
    double cont = (K.C.kappagrey[mgi] * K.C.rho[mgi]);
    cont = cont * p.e_rf * dist * (1. - (2. * dot(vel_vec, p.dir) / ARTIS_CLIGHT));
    safeadd(&K.E.rpkt_emiss[mgi], 1.e-20 * cont);
  }
}

// rpkt.cc:623-700: the step's draw, boundary and the cases without a line walk; RSTEP_WALK when get_event's walk is
// set up in S, RSTEP_END when the step's end can run (rpkt_step_finish), RSTEP_DONE after an error
DEVFN int rpkt_step_begin(Tx &x, Pkt &p, double t2, RStep &S) {
  const Ctx &K = x.K;
  const int npm = K.G.npts_model;
  S.mgi = cell_mgi(K, p.where);
  S.oldmgi = S.mgi;
  lwork(x.L, WK_RPKT_STEPS, 1);
  const double zrand = artis_rng_uniform_pos(&x.rng);
  const double tau_next = -1. * log(zrand);
  S.snext = -1;
  S.sdist = boundary_cross(x, p, &S.snext);
  STAMP(x, 0);
  S.cross0 = (S.sdist == 0);
  S.find_nextline = false;
  S.eventtype = -1;
  if (S.cross0) return RSTEP_END;
  const double maxsdist = max_sdist(K, p, S.sdist);
  if (S.sdist > maxsdist) {
    x.err(ERR_SDIST, p.number, p.where);
    return RSTEP_DONE;
  }
  if (((S.snext != -99) && (S.snext < 0)) || (S.snext >= K.G.ngrid)) {
    x.err(ERR_BADCELL, p.number, S.snext);
    return RSTEP_DONE;
  }
  if (S.sdist > K.R.max_path_step) {
    S.sdist = K.R.max_path_step;
    S.snext = p.where;
  }
  S.tdist = (t2 - p.prop_time) * ARTIS_CLIGHT_PROP;
  S.kap.nu = 0.;
  S.kap.total = S.kap.es = S.kap.ff = S.kap.bf = S.kap.ffheating = 0.;
  const int mgi = S.mgi;
  S.k = (mgi == npm) ? -1 : K.C.ne_index[mgi];
  if (mgi == npm) {
    S.edist = DBL_MAX;
    S.find_nextline = true;
    return RSTEP_END;
  }
  if (K.C.thick[mgi] == 1) {
    // grey optically thick cell: electron scattering only (rpkt.cc:697-703); no continuum opacity is evaluated,
    // so the estimator terms of this step use kappa = 0 (deviation D7)
    const double kappa = K.C.kappagrey[mgi] * K.C.rho[mgi] * doppler_packet(K, p);
    S.edist = (tau_next - 0.0) / kappa;
    S.find_nextline = true;
    return RSTEP_END;
  }
  if (get_event_begin(x, S.k, mgi, p, S, tau_next, fmin(S.tdist, S.sdist))) return RSTEP_WALK;
  return x.ok ? RSTEP_END : RSTEP_DONE;
}

// rpkt.cc:700-813: the end of the step from S (the event distance and type, or the immediate cell change)
template <typename Cold>
DEVFN bool rpkt_step_finish(Tx &x, Pkt &p, double t2, RStep &S, const Cold &cold) {
  const Ctx &K = x.K;
  const int npm = K.G.npts_model;
  int mgi = S.mgi;
  const int oldmgi = S.oldmgi;
  // One inlined copy each of the cell change and of the move / estimator / move sequence, shared by the ways a
  // step ends (the register pressure of k_rpkt grows with every inlined copy): cross = change cell (sdist == 0
  // at once, or a step that ends on the boundary of another cell), boundary_step = the step ended on the boundary.
  bool cross = S.cross0, boundary_step = false;
  const bool find_nextline = S.find_nextline;
  if (!cross) {
    const double sdist = S.sdist, tdist = S.tdist, edist = S.edist;
    if (!(edist >= 0)) {
      x.err(ERR_EDIST, p.number, 0);
      return false;
    }
    // which distance ends the step (rpkt.cc:711-806: boundary, event, end of timestep)
    int which;
    double dist;
    if ((sdist < tdist) && (sdist < edist)) {
      which = 0;
      dist = sdist;
    } else if ((edist < sdist) && (edist < tdist)) {
      which = 1;
      dist = edist;
    } else if ((tdist < sdist) && (tdist < edist)) {
      which = 2;
      dist = tdist;
    } else {
      x.err(ERR_NOEVENT, p.number, 1);
      return false;
    }
    move_pkt_withtime(K, p, dist / 2.);
    update_estimators(x, p, S.kap, dist);
    if (K.R.do_rlc_est == 1 || K.R.do_rlc_est == 2) rlc_emiss_rpkt(K, p, dist);
    if (which == 2) {
      p.prop_time = t2;
      move_pkt(K, p, dist / 2.);
      p.last_event = p.last_event + 1000;
      if (find_nextline) closest_transition_empty(K, p);
      return false;
    }
    move_pkt_withtime(K, p, dist / 2.);
    STAMP(x, 3);
    if (which == 1) {
      const int k = S.k;
      if (K.C.thick[mgi] == 1)
        cold(x, p, [&](Tx &tx, Pkt &tp) { rpkt_event_thickcell(tx, tp); });
      else if (S.eventtype == ARTIS_RPKT_EVENTTYPE_BB)
        rpkt_event_boundbound(x, p);
      else if (S.eventtype == ARTIS_RPKT_EVENTTYPE_CONT)
        cold(x, p, [&](Tx &tx, Pkt &tp) {
          const Kappa kc = S.kap;
          rpkt_event_continuum(tx, tp, kc, k, mgi);
        });
      else
        x.err(ERR_NOEVENT, p.number, 0);
      return (x.ok && p.type == ARTIS_TYPE_RPKT && (mgi == npm || mgi == oldmgi));
    }
    boundary_step = true;
    cross = (S.snext != p.where);
  }
  if (cross) {
    change_cell(x, p, S.snext);
    mgi = cell_mgi(K, p.where);
  }
  if (boundary_step) {
    p.scat_count = 0;
    p.last_event = p.last_event + 100;
    if (find_nextline) {
      if (mgi != npm && K.C.thick[mgi] != 1) closest_transition_empty(K, p);
    }
  }
  return (p.type == ARTIS_TYPE_RPKT && (mgi == npm || mgi == oldmgi));
}

// rpkt.cc:623-813, the whole step; true while the packet stays an r-packet in the same cell
template <typename Cold = ColdFull>
DEVFN bool do_rpkt_step(Tx &x, Pkt &p, double t2, const Cold &cold = Cold()) {
  RStep S;
  int r = rpkt_step_begin(x, p, t2, S);
  if (r == RSTEP_WALK) {
    get_event_walk(x, p, S, 1 << 30);
    r = x.ok ? RSTEP_END : RSTEP_DONE;
  }
  return r == RSTEP_END ? rpkt_step_finish(x, p, t2, S, cold) : false;
}

// ------------------------------------------------------------------------------------------ fb emission
// ratecoeff.cc:263-279
DEVFN double alpha_sp_E_integrand(const Ctx &K, const float *xs, double nu_edge, float T, double nu) {
  const float sigma_bf = (float)photoionization_crosssection_fromtable(K, xs, nu_edge, nu);
  return ARTIS_TWOOVERCLIGHTSQUARED * sigma_bf * pow(nu, 3) / nu_edge * exp(-ARTIS_HOVERKB * nu / T);
}
DEVFN double alpha_sp_piece(const Ctx &K, const float *xs, double nu_threshold, float T, double a, double half) {
  const double gx[4] = {-0.8611363115940526, -0.3399810435848563, 0.3399810435848563, 0.8611363115940526};
  const double gw[4] = {0.3478548451374538, 0.6521451548625461, 0.6521451548625461, 0.3478548451374538};
  const double mid = a + half;
  double s = 0.;
  for (int q = 0; q < 4; q++) s += gw[q] * alpha_sp_E_integrand(K, xs, nu_threshold, T, mid + half * gx[q]);
  return s * half;
}
// ratecoeff.cc:628-684 with deviation D3 (see oracle/oracle.cc), for the draw zrand = 1 - uniform
DEVFN double select_continuum_nu_z(const Ctx &K, int e, int lowerion, int lower, int upperionlevel, float T_e,
                                   double zrand) {
  int target = 0;
  for (int t = 0; t < get_nphixstargets(K, e, lowerion, lower); t++)
    if (get_phixsupperlevel(K, e, lowerion, lower, t) == upperionlevel) {
      target = t;
      break;
    }
  const double E_threshold = get_phixs_threshold(K, e, lowerion, lower, target);
  const double nu_threshold = ARTIS_ONEOVERH * E_threshold;
  const double nu_max_phixs = nu_threshold * K.T.last_phixs_nuovernuedge;
  const int npieces = K.T.nphixspoints;
  const float *xs = level_photoion_xs(K, e, lowerion, lower);
  const double deltanu = (nu_max_phixs - nu_threshold) / npieces;
  const double half = 0.5 * deltanu;
  double head = 0.;
  for (int j = 0; j < npieces; j++) head += alpha_sp_piece(K, xs, nu_threshold, T_e, nu_threshold + j * deltanu, half);
  const double total_alpha_sp = head;
  double alpha_sp_old = total_alpha_sp;
  double alpha_sp = total_alpha_sp;
  head = 0.;
  int i;
  for (i = 1; i < npieces; i++) {
    alpha_sp_old = alpha_sp;
    head += alpha_sp_piece(K, xs, nu_threshold, T_e, nu_threshold + (i - 1) * deltanu, half);
    alpha_sp = total_alpha_sp - head;
    if (zrand >= alpha_sp / total_alpha_sp) break;
  }
  const double nuoffset = (total_alpha_sp * zrand - alpha_sp_old) / (alpha_sp - alpha_sp_old) * deltanu;
  return nu_threshold + (i - 1) * deltanu + nuoffset;
}

// the same with its draw (the reference's order: the draw first)
DEVNI double select_continuum_nu(Tx &x, int e, int lowerion, int lower, int upperionlevel, float T_e) {
  const double zrand = 1. - artis_rng_uniform(&x.rng);
  return select_continuum_nu_z(x.K, e, lowerion, lower, upperionlevel, T_e, zrand);
}

// select_continuum_nu's integral for every lane of the wave that asks for one (want; every lane of the wave calls
// this, convergent).  The requests are taken one continuum at a time: the lanes evaluate the continuum's npieces
// quadrature pieces in parallel (pieces q, q + 64, ...; the same alpha_sp_piece values as the serial loops), one
// pass adds them in the reference's order into the running sums P[i] (pieces 0 .. i-1) in the wave's LDS slot P,
// and every lane asking for that continuum at the same T_e then finds its own frequency by a binary search over
// them with its own draw.  alpha_sp after i pieces is total - P[i] and the reference's test zrand >= alpha_sp /
// total flips once along i (the pieces are non-negative, so the rounded sums only grow), so the search stops where
// the serial loop breaks and the result is select_continuum_nu's bit for bit.  zrand is the lane's draw (1 -
// uniform, drawn by the caller where select_continuum_nu draws it).  A one-zone model's deactivations share a few
// continua, so the serial pass is paid once per continuum and wave pass instead of twice per request.
#define WAVE_FB_MAXR 4  // pieces per lane held in registers (npieces <= 256; more: evaluated in the serial pass)
#define WAVE_FB_MAXP 256  // pieces whose running sums fit the LDS slot (more: the serial search per request)
typedef __attribute__((address_space(3))) double lds_double;
DEVFN double wave_select_continuum_nu(const Ctx &K, bool want, int e, int lowerion, int lower, int upperionlevel,
                                      float T_e, double zrand, lds_double *P) {
  double result = 0.;
  bool todo = want;
  unsigned long long m = __ballot(todo);
  const int lane = (int)__lane_id();
  while (m) {
    const int ld = __ffsll((long long)m) - 1;
    const int le = __builtin_amdgcn_readlane(e, ld), li = __builtin_amdgcn_readlane(lowerion, ld);
    const int ll = __builtin_amdgcn_readlane(lower, ld), lu = __builtin_amdgcn_readlane(upperionlevel, ld);
    const int lTb = __builtin_amdgcn_readlane(__float_as_int(T_e), ld);
    const float lT = __int_as_float(lTb);
    int target = 0;
    for (int t = 0; t < get_nphixstargets(K, le, li, ll); t++)
      if (get_phixsupperlevel(K, le, li, ll, t) == lu) {
        target = t;
        break;
      }
    const double E_threshold = get_phixs_threshold(K, le, li, ll, target);
    const double nu_threshold = ARTIS_ONEOVERH * E_threshold;
    const double nu_max_phixs = nu_threshold * K.T.last_phixs_nuovernuedge;
    const int npieces = K.T.nphixspoints;
    const float *xs = level_photoion_xs(K, le, li, ll);
    const double deltanu = (nu_max_phixs - nu_threshold) / npieces;
    const double half = 0.5 * deltanu;
    double pc[WAVE_FB_MAXR];
#pragma unroll
    for (int r = 0; r < WAVE_FB_MAXR; r++) {
      const int j = lane + 64 * r;
      pc[r] = (j < npieces) ? alpha_sp_piece(K, xs, nu_threshold, lT, nu_threshold + j * deltanu, half) : 0.;
    }
    auto piece = [&](int j) {  // piece j from its lane (j wave-uniform); past the registers, evaluated here
      if (npieces > 64 * WAVE_FB_MAXR) return alpha_sp_piece(K, xs, nu_threshold, lT, nu_threshold + j * deltanu, half);
      double v = 0.;
#pragma unroll
      for (int r = 0; r < WAVE_FB_MAXR; r++)
        if ((j >> 6) == r) v = readlane_d(pc[r], j & 63);
      return v;
    };
    // the lanes served by this pass: the same continuum at the same temperature (or only the first, when the running
    // sums do not fit the LDS slot)
    const bool shared = npieces >= 2 && npieces <= WAVE_FB_MAXP;
    const bool same = todo && (shared ? (e == le && lowerion == li && lower == ll && upperionlevel == lu &&
                                         __float_as_int(T_e) == lTb)
                                      : lane == ld);
    if (shared) {
      double head = 0.;
      if (lane == 0) P[0] = 0.;
      for (int j = 0; j < npieces; j++) {
        head += piece(j);
        if (lane == 0) P[j + 1] = head;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const double total = head;
      if (same) {
        // the serial loop breaks at the first i in [1, npieces) with zrand >= (total - P[i]) / total
        int lo = 1, hi = npieces;
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if (zrand >= (total - P[mid]) / total)
            hi = mid;
          else
            lo = mid + 1;
        }
        // (no break: the loop ends with i = npieces, alpha_sp_old and alpha_sp of pieces npieces - 2 and npieces - 1)
        const int i = lo, k = (i == npieces) ? npieces - 1 : i;
        const double alpha_sp_old = total - P[k - 1], alpha_sp = total - P[k];
        const double nuoffset = (total * zrand - alpha_sp_old) / (alpha_sp - alpha_sp_old) * deltanu;
        result = nu_threshold + (i - 1) * deltanu + nuoffset;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();  // (the slot's readers are done before the next continuum's sums)
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    } else {
      const double lz = readlane_d(zrand, ld);
      double head = 0.;
      for (int j = 0; j < npieces; j++) head += piece(j);
      const double total_alpha_sp = head;
      double alpha_sp_old = total_alpha_sp;
      double alpha_sp = total_alpha_sp;
      head = 0.;
      int i;
      for (i = 1; i < npieces; i++) {
        alpha_sp_old = alpha_sp;
        head += piece(i - 1);
        alpha_sp = total_alpha_sp - head;
        if (lz >= alpha_sp / total_alpha_sp) break;
      }
      const double nuoffset = (total_alpha_sp * lz - alpha_sp_old) / (alpha_sp - alpha_sp_old) * deltanu;
      if (lane == ld) result = nu_threshold + (i - 1) * deltanu + nuoffset;
    }
    m &= ~__ballot(same);
    todo = todo && !same;
  }
  return result;
}

// ------------------------------------------------------------------------------------------ macro-atom
// first j in [0, n) with cum[j] > x (n if none): the reference's `rate += individ[j]; if (x < rate) break;`
// scan, exact because cum holds those running sums in the same order (non-decreasing)
DEVFN int first_above(const double *cum, int n, double x, unsigned long long &probes) {
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    probes++;
    if (cum[mid] > x)
      hi = mid;
    else
      lo = mid + 1;
  }
  return lo;
}
// One macro-atom is walked jump by jump and its deactivation applied to the packet afterwards
// (ma_finish).  The megakernel calls both back to back (do_macroatom); the wavefront engine runs the walk in a
// lean kernel that never loads the 304-byte record and defers ma_finish to the kernel the packet moves to.
enum { MA_CONTINUE = 0, MA_END_BB = 1, MA_END_COLDEEXC = 2, MA_END_COLRECOMB = 3, MA_END_FB = 4, MA_FAILED = -1,
       MA_DEFER = -2, MA_PENDING = -3 };
// WaveState::pend code of a walk parked between jumps (.y = unique level it stands on): set when a jump of the
// cached walk needs the exact sums (k_ma_exact), read when the walk resumes in k_ma
#define MA_RESUME 16
struct MaEnd {
  int code, ion, a, b;  // BB: a = line, b = unique index of the emitting level;
                        // FB: a = level of the lower ion, b = unique index of the recombining level
};

// The cached walk in its lean form: lane state = (unique level, cell, record line).  Per jump: the level's
// 32-byte MaMeta (L2-resident table) and its compact key record (DevCells::ma_key): the 9 action keys, then a
// binary search over the keys of the selected action -- for the internal same-ion jumps (most jumps) on the
// record's first 128-byte line, or via its separators there and one 64-key block line -- and one 8-byte load of
// the target (level, record offset).  A comparison the 32-bit keys cannot decide sends the jump to ma_jump_exact,
// which recomputes the reference's exact sums; the selections -- and so the RNG draws and every result -- are the
// reference's linear scans over its running sums (macroatom.cc:502-525 and the do_macroatom_* searches).
struct MaLaneC {
  int ul, k;
  uint32_t line;    // first 128-byte line of the current level's record in DevCells::ma_key (MA_NOLINE: none)
  int32_t rowline;  // row mode: the first line of the cell's row; -1: level mode (DevCells::ma_lptr)
  unsigned jumps;
  unsigned long long ntrans;
};
// The context fields a macro-atom jump reads, held in scalar registers by k_ma (ma_hot(*ctxp): loaded once from the
// device context at kernel entry).  Read from the context copy in LDS instead, every use was an LDS load whose
// result the compiler re-read after the kernel's LDS stores (the record-line staging), a dependent LDS round trip
// in front of the jump's global loads; the pointers also lived in vector registers.
struct MaHot {
  const uint16_t *ma_key;
  const MaMeta *ma_meta;
  const MaWalk *ma_walk;
  const int2 *down_target, *up_target;
  const uint32_t *ma_lptr;
  uint32_t *ma_lhist;
  int32_t nlevels_total;
};
DEVFN MaHot ma_hot(const Ctx &K) {
  return MaHot{K.C.ma_key,   K.T.ma_meta, K.T.ma_walk,    K.T.down_target,
               K.T.up_target, K.C.ma_lptr, K.C.ma_lhist, K.T.nlevels_total};
}
// the record line of level ul (MaMeta::rec_off rec_off) in the walk's cell
DEVFN uint32_t ma_line(const MaHot &H, int32_t rowline, int k, int ul, int rec_off) {
  if (rowline >= 0) return (uint32_t)rowline + ((uint32_t)rec_off >> 6);
  return H.ma_lptr ? H.ma_lptr[(int64_t)k * H.nlevels_total + ul] : MA_NOLINE;
}
DEVFN uint32_t ma_line(const Ctx &K, int32_t rowline, int k, int ul, int rec_off) {
  return ma_line(ma_hot(K), rowline, k, ul, rec_off);
}
DEVFN int32_t ma_rowline(const Ctx &K, int k) {
  const int row = K.C.ma_row[k];
  return row >= 0 ? (int32_t)(((int64_t)row * K.C.ma_key_stride) >> 6) : -1;
}
DEVFN void ma_set_level(const MaHot &H, MaLaneC &m, int ul) {
  m.ul = ul;
  m.line = ma_line(H, m.rowline, m.k, ul, H.ma_meta[ul].rec_off);
}
DEVFN void ma_set_level(const Ctx &K, MaLaneC &m, int ul) { ma_set_level(ma_hot(K), m, ul); }

// the outcome of selecting transition j (reference list order) of action sel at level ul: MA_CONTINUE with the
// lane moved to the target level, or a deactivation in `end` (macroatom.cc:174-414)
DEVFN int ma_apply_selection(const Ctx &K, const MaHot &H, const LocalCounters &L, MaLaneC &m, MaEnd &end, int sel,
                             int j, int doff, int uoff, int base_lower) {
  const int ul = m.ul;
  switch (sel) {
    case ARTIS_MA_ACTION_INTERNALDOWNSAME:
      ma_set_level(H, m, K.T.ion_uniqueleveloffset[K.T.level_ui[ul]] + K.T.line_lower[K.T.downtrans_lineindex[doff + j]]);
      return MA_CONTINUE;
    case ARTIS_MA_ACTION_INTERNALUPSAME:
      ma_set_level(H, m, K.T.ion_uniqueleveloffset[K.T.level_ui[ul]] + K.T.line_upper[K.T.uptrans_lineindex[uoff + j]]);
      return MA_CONTINUE;
    case ARTIS_MA_ACTION_RADDEEXC:
      // the line index is looked up by ma_finish (end.a = -1 - downtrans slot): a load here would hold the whole
      // wave of k_ma for a round trip in most passes (some lane deactivates radiatively in ~2/3 of them)
      end.code = MA_END_BB;
      end.ion = 0;
      end.a = -1 - (doff + j);
      end.b = ul;
      return MA_END_BB;
    case ARTIS_MA_ACTION_RADRECOMB:
      end.code = MA_END_FB;
      end.ion = 0;
      end.a = j;
      end.b = ul;
      return MA_END_FB;
    case ARTIS_MA_ACTION_INTERNALDOWNLOWER:
      lctr(L, CTR_MA_STAT_INTERNALDOWNLOWER);
      ma_set_level(H, m, base_lower + j);
      return MA_CONTINUE;
    default: {  // INTERNALUPHIGHER (macroatom.cc:382-414)
      lctr(L, CTR_MA_STAT_INTERNALUPHIGHER);
      const int ui = K.T.level_ui[ul];
      ma_set_level(H, m, K.T.ion_uniqueleveloffset[ui + 1] + K.T.phixstarget_levelindex[K.T.level_phixstargets_offset[ul] + j]);
      return MA_CONTINUE;
    }
  }
}

// macroatom.cc:866-884 for the cached walk: the upper ion from the Auger-electron probabilities, its ground level
DEVFN int ma_apply_nt(const Ctx &K, const LocalCounters &L, artis_rng &rng, MaLaneC &m, int number) {
  lctr(L, CTR_MA_STAT_INTERNALUPHIGHERNT);
  const int ui = K.T.level_ui[m.ul];
  const int e = K.T.ion_element[ui];
  const int ion = ui - K.T.elem_uniqueionoffset[e];
  const int upperion = nt_random_upperion(K, rng, K.C.ne_mgi[m.k], e, ion, false);
  if (upperion < 0) {
    fail(K, ERR_MA_SELECT, number, 9);
    return MA_FAILED;
  }
  ma_set_level(K, m, K.T.ion_uniqueleveloffset[ui + upperion - ion]);
  return MA_CONTINUE;
}

// One jump of the cached walk with the reference's exact double sums, recomputed from the cell tables through
// ma_foreach_rate (the very sums k_marates condensed into keys): macroatom.cc:502-525 and the transition search of
// the selected action.  Draws zrand (and zr) itself; runs where a key comparison was undecided (k_ma_exact,
// do_macroatom), with the lane's RNG counter reset to the start of the jump.
DEVNI int ma_jump_exact(const Ctx &K, const LocalCounters &L, artis_rng &rng, MaLaneC &m, MaEnd &end, int number,
                        double t_mid) {
  m.jumps++;
  const int ul = m.ul, k = m.k;
  const int mgi = K.C.ne_mgi[k];
  const MaMeta mm = K.T.ma_meta[ul];
  const double *pops = K.C.pops + (int64_t)k * K.T.nlevels_total;
  const double *corr = K.C.corrphot + (int64_t)k * K.T.ntargets_total;
  auto pop = [&](int u) { return pops[u]; };
  auto cph = [&](int slot) { return corr[slot]; };
  double pr[ARTIS_MA_ACTION_COUNT];
  for (int a = 0; a < ARTIS_MA_ACTION_COUNT; a++) pr[a] = 0.;
  ma_foreach_rate(K, mgi, ul, t_mid, pop, cph, [&](int kind, int j, double R, double C, double et, double eg, double ec) {
    ma_accumulate(pr, kind, R, C, et, eg, ec);
    return false;
  });
  pr[ARTIS_MA_ACTION_INTERNALUPHIGHERNT] = ma_nt_total(K, mgi, ul);
  double total_transitions = 0.;
  for (int a = 0; a < ARTIS_MA_ACTION_COUNT; a++) total_transitions += pr[a];
  double zrand, zr;
  artis_rng_jump_pair(&rng, &zrand, &zr);  // (the action draw and the transition draw)
  rng.n++;
  const double randomrate = zrand * total_transitions;
  double rate = 0.;
  int sel = ARTIS_MA_ACTION_COUNT;
  for (int a = 0; a < ARTIS_MA_ACTION_COUNT; a++) {
    rate += pr[a];
    if (rate > randomrate) {
      sel = a;
      break;
    }
  }
  if (rate <= randomrate) {
    fail(K, ERR_MA_RANDOM, number, ul);
    return MA_FAILED;
  }
  if (sel == ARTIS_MA_ACTION_COLDEEXC || sel == ARTIS_MA_ACTION_COLRECOMB) {
    end.code = (sel == ARTIS_MA_ACTION_COLDEEXC) ? MA_END_COLDEEXC : MA_END_COLRECOMB;
    end.ion = end.a = end.b = 0;
    return end.code;
  }
  if (sel == ARTIS_MA_ACTION_INTERNALUPHIGHERNT) return ma_apply_nt(K, L, rng, m, number);
  // the transition: first running sum of action sel above zr * total, in the reference's list order
  rng.n++;
  const double x = zr * pr[sel];
  const int kind = (sel == ARTIS_MA_ACTION_RADDEEXC || sel == ARTIS_MA_ACTION_INTERNALDOWNSAME) ? MA_KIND_DOWN
                   : (sel == ARTIS_MA_ACTION_RADRECOMB || sel == ARTIS_MA_ACTION_INTERNALDOWNLOWER) ? MA_KIND_RECOMB
                   : (sel == ARTIS_MA_ACTION_INTERNALUPSAME) ? MA_KIND_UP
                                                             : MA_KIND_UPHIGHER;
  double run[ARTIS_MA_ACTION_COUNT];
  for (int a = 0; a < ARTIS_MA_ACTION_COUNT; a++) run[a] = 0.;
  int found = -1;
  ma_foreach_rate(K, mgi, ul, t_mid, pop, cph, [&](int kd, int j, double R, double C, double et, double eg, double ec) {
    ma_accumulate(run, kd, R, C, et, eg, ec);
    if (kd == kind) m.ntrans++;
    if (kd == kind && run[sel] > x) {
      found = j;
      return true;
    }
    return false;
  });
  if (found < 0) {
    fail(K, ERR_MA_SELECT, number, 10 + sel);
    return MA_FAILED;
  }
  return ma_apply_selection(K, ma_hot(K), L, m, end, sel, found, mm.doff, mm.uoff, mm.base_lower);
}

// MA_DEFER: a key comparison was undecided; the jump has not happened (m.jumps unchanged) and the caller resets
// the RNG counter to its value before the call and runs ma_jump_exact.
// line != nullptr (k_ma): the lane's 128-byte LDS slot, laid out chunk-major for the wave ([8][64] 16-byte
// chunks, lane-linear per chunk), already holding the first line of the record (positions 0..63: the action keys
// and, for ~99% of levels, both same-ion trees), fetched for the whole wave by ma_fetch_lines; the tree search
// then probes LDS instead of making one dependent trip to the cache hierarchy per tree level.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) u32x4 lds_uint4;
typedef __attribute__((address_space(3))) uint16_t lds_u16;
typedef const __attribute__((address_space(1))) u32x4 glb_uint4;

// Wave-cooperative fetch of one 128-byte line per lane (line index `myline` in units of 128 bytes from `base`; a lane
// without a line names line 0) into the wave's chunk-major LDS image wl[chunk * 64 + lane].  Instruction i has lanes
// 8j..8j+7 read the eight 16-byte chunks of the line of lane 8i + j, so each load instruction touches 8 lines
// instead of 64.  The memory system's rate is set by the (instruction, line) pairs it serves: random 128-byte
// lines fetched this way arrive at 45 G lines/s (5.8 TB/s) on MI355X against 9.7 G lines/s (1.24 TB/s) when every
// lane loads its own line (tools/linerate.hip, profiles/r02_linerate.txt).  Wave-uniform control flow only.
struct WaveLines {
  u32x4 c[8];
};
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) uint64_t lds_u64;
#ifndef ARTIS_MA_FETCH_ADDR
#define ARTIS_MA_FETCH_ADDR 0
#endif
#if ARTIS_MA_FETCH_ADDR
// xa: the wave's 64-entry LDS exchange slot for the lines' byte addresses (lane L's at (L & 7) * 8 + (L >> 3), so
// that the eight addresses a lane loads for are contiguous).  Each lane forms its own line's 64-bit address once; a
// reader adds its chunk offset, one 64-bit add per line (A/B: no faster than exchanging indices, the default)
DEVFN void wave_fetch_issue(const void *base, uint32_t myline, WaveLines &w, lds_u64 *xa) {
  const int lane = (int)__lane_id();
  xa[(lane & 7) * 8 + (lane >> 3)] = (uint64_t)(uintptr_t)base + ((uint64_t)myline << 7);
  __builtin_amdgcn_wave_barrier();
  const lds_uint4 *xr = (const lds_uint4 *)(xa + 8 * (lane >> 3));
  const u32x4 a0 = xr[0], a1 = xr[1], a2 = xr[2], a3 = xr[3];
  const uint64_t ad[8] = {a0.x | (uint64_t)a0.y << 32, a0.z | (uint64_t)a0.w << 32, a1.x | (uint64_t)a1.y << 32,
                          a1.z | (uint64_t)a1.w << 32, a2.x | (uint64_t)a2.y << 32, a2.z | (uint64_t)a2.w << 32,
                          a3.x | (uint64_t)a3.y << 32, a3.z | (uint64_t)a3.w << 32};
  const uint64_t coff = (uint64_t)(lane & 7) * 16;
#pragma unroll
  for (int i = 0; i < 8; i++)
    w.c[i] = *(glb_uint4 *)(uintptr_t)(ad[i] + coff);  // (an idle lane names line 0)
}
#else
// xi: the wave's 64-word LDS exchange slot for the line indices (lane L's index at (L & 7) * 8 + (L >> 3), so
// that the eight indices a lane loads for are contiguous: one write, two 16-byte reads, one wait)
DEVFN void wave_fetch_issue(const void *base, uint32_t myline, WaveLines &w, lds_u64 *xa) {
  const int lane = (int)__lane_id();
  lds_u32 *xi = (lds_u32 *)xa;
  glb_uint4 *g = (glb_uint4 *)base;
  xi[(lane & 7) * 8 + (lane >> 3)] = myline;
  __builtin_amdgcn_wave_barrier();
  const u32x4 i0 = ((lds_uint4 *)xi)[2 * (lane >> 3)], i1 = ((lds_uint4 *)xi)[2 * (lane >> 3) + 1];
  const uint32_t ls[8] = {i0.x, i0.y, i0.z, i0.w, i1.x, i1.y, i1.z, i1.w};
#pragma unroll
  for (int i = 0; i < 8; i++) w.c[i] = g[(size_t)ls[i] * 8 + (lane & 7)];  // (an idle lane names line 0)
}
#endif
DEVFN void wave_fetch_commit(const WaveLines &w, lds_uint4 *wl) {
  const int lane = (int)__lane_id();
#pragma unroll
  for (int i = 0; i < 8; i++) wl[(lane & 7) * 64 + 8 * i + (lane >> 3)] = w.c[i];  // idle lanes' slots: unread
  __builtin_amdgcn_wave_barrier();
}

// a load through the global address space (global_load, counted by vmcnt only; a flat load also holds lgkmcnt)
template <typename T>
DEVFN T gload(const T *p) {
  return *(const __attribute__((address_space(1))) T *)p;
}

// the level's MaWalk words the cached walk reads (engine_dev.h): w0 = (nd | nu << 16, doff, uoff, base_lower),
// w1 = the packed record layout.  (Until round 6 this was MaMeta's (doff, uoff, base_lower), (nd, nu, nr, nt), and every
// step worked out ma_layout from the counts.)
struct MaMetaW {
  int4 w0, w1;
};
DEVFN MaMetaW ma_walk_load(const MaWalk *ma_walk, int ul) {
  glb_uint4 *mp = (glb_uint4 *)(ma_walk + ul);
  const u32x4 a = mp[0], b = mp[1];
  return MaMetaW{make_int4((int)a.x, (int)a.y, (int)a.z, (int)a.w), make_int4((int)b.x, (int)b.y, (int)b.z, (int)b.w)};
}
DEVFN MaMetaW ma_walk_load(const Ctx &K, int ul) { return ma_walk_load(K.T.ma_walk, ul); }

// The cached walk as a resumable per-pass step (k_ma).  In SIMT every pass of a wave lasts as long as its slowest
// lane; a search that probed record lines other than the staged one made one dependent trip to memory per probe,
// and nearly every pass of a 64-lane wave waited for some lane doing that (profiles/r02_ma_phase_stamps.txt).
// Here a search that needs a line other than the one staged in the lane's LDS slot stops (MA_PENDING) and names
// that line (pline); the next pass fetches it with everybody else's lines (wave_fetch_issue) and the search
// resumes where it stopped.  With the two-level record layout (engine_dev.h ma_layout) a jump needs at most two
// lines.  Every comparison is decided exactly as by ma_key_cmp, so the selections -- and every result -- are the
// uncached walk's.
//
// Key comparisons in integers: qh = the high 16 bits of floor(q).  A key whose high half is below qh lies at
// least 1 below q (decided "not greater"); above qh + 1, at least 65536 above q (decided "greater"); only a high
// half of qh or qh + 1 needs the low half and the banded comparison ma_key_cmp (~2 in 65536 comparisons).
DEVFN uint32_t ma_qh(double q) { return ((uint32_t)q) >> 16; }
// The walk's draws stay Philox words (artis_rng_jump_words) until a comparison needs the value itself:
// q = z * MA_KEY_SCALE (z = artis_rng_word_unit(lo, hi), the reference-order expression), and a lower bound of its
// high half from the word hi alone.  With T = hi = floor(m / 2^21) for the draw's 53-bit integer m, the exact
// product m (2^32 - 1) / 2^53 lies in (T - 1, T + 1), and its double rounding moves it by less than 2^-21, so
// floor(q) is T - 2, T - 1 or T and ma_qh_draw <= ma_qh(q) <= ma_qh_draw + 1.  A lower qh is still exact: it can
// only be ma_qh(q) - 1 when q lies less than 3 above a multiple of 65536, so every high half it decides (below qh, or
// above qh + 1) is decided the same way by ma_qh(q), and every other goes to the banded comparison with q as before
// -- the same selections and the same undecided (deferred) jumps, without the conversions to double per jump.
DEVFN uint32_t ma_qh_draw(uint32_t hi) { return (hi < 2u ? 0u : hi - 2u) >> 16; }
DEVFN double ma_q_draw(uint32_t lo, uint32_t hi) { return artis_rng_word_unit(lo, hi) * MA_KEY_SCALE; }

#ifdef ARTIS_STAMPS
// diagnostic build: per selected action, [a] searches, [16 + a] MA_PENDING returns, [32 + a] probes
__device__ unsigned long long g_ma_diag[48];
#define MA_DIAG(i)                             \
  do {                                         \
    if (L.diag) atomicAdd(&L.diag[i], 1ull); \
  } while (0)
#else
#define MA_DIAG(i) \
  do {             \
  } while (0)
#endif

struct MaLaneR : MaLaneC {
  uint32_t n0;         // RNG counter at the start of the jump in progress (the caller's reset point for MA_DEFER)
  int sel;             // -1: the next step starts a jump; otherwise the action whose transition search is pending
  int pline;           // record line (64 key positions) staged for this step
  int lo, hi, end;     // binary search in progress over entries [lo, hi) of a range of `end` entries ...
  int base;            // ... at record positions base + i
  int blk;             // same-ion array in blocks: -1 while its separators are searched, then the block
  uint32_t q2lo, q2hi;  // the transition draw's Philox words (its value on the key scale: ma_q_draw)
  uint32_t q2h;
};

// ---- the jump of a walk whose (cell, level) has no key record (level mode), made by the whole wave ------------
#define MA_COOP_RANDOM (-1)  // the action draw exceeds the total (the reference's abort, ERR_MA_RANDOM)
#define MA_COOP_NOSEL (-2)   // no entry of the action's list exceeds the transition draw (ERR_MA_SELECT)
// The jump of a walk whose (cell, level) pair has no key record.  The action comes from the pair's exact totals
// (DevCells::marates, the sums of ma_foreach_rate in the reference's order, macroatom.cc:502-525), drawn by each such
// lane itself (ma_coop_action); only a transition action's list search is made by the whole wave (ma_coop_search).
// ma_coop_action returns the action (or MA_COOP_RANDOM) and *x = z2 times the action's total, the search's target.
DEVFN int ma_coop_action(const Ctx &K, int k, int ul, double z1, double z2, double *x) {
  const double *tot = K.C.marates + ((int64_t)k * K.T.nlevels_total + ul) * ARTIS_MA_ACTION_COUNT;
  double pr[ARTIS_MA_ACTION_COUNT];
  double total = 0.;
  for (int a = 0; a < ARTIS_MA_ACTION_COUNT; a++) {
    pr[a] = tot[a];
    total += pr[a];
  }
  const double randomrate = z1 * total;
  double rate = 0.;
  int sel = MA_COOP_RANDOM;
  for (int a = 0; a < ARTIS_MA_ACTION_COUNT; a++) {
    rate += pr[a];
    if (rate > randomrate) {
      sel = a;
      break;
    }
  }
  double xs = 0.;
#pragma unroll
  for (int a = 0; a < ARTIS_MA_ACTION_COUNT; a++)
    if (a == sel) xs = z2 * pr[a];
  *x = xs;
  return sel;
}
DEVFN bool ma_coop_needs_search(int sel) {
  return sel >= 0 && sel != ARTIS_MA_ACTION_COLDEEXC && sel != ARTIS_MA_ACTION_COLRECOMB &&
         sel != ARTIS_MA_ACTION_INTERNALUPHIGHERNT;
}
// Wave-uniform: every lane calls it with the same (k, ul, sel, x) and gets the same entry of action sel's list:
// the lanes evaluate 64 individual rates at a time (ma_rate_at: the expressions the totals were summed from) and
// the running sum is added in list order, one term per step, read from the evaluating lane's register (v_readlane)
// -- the reference's linear scan (do_macroatom_raddeexcitation etc.), the same double sums as ma_jump_exact.
// Returns sel, *j the entry (or MA_COOP_NOSEL).
// (out of line: inlined into k_ma, its rate expressions would raise the register allocation of the whole walk)
#ifdef ARTIS_MA_COOP_INLINE
DEVFN
#else
DEVNI
#endif
int ma_coop_search(const Ctx &K, int k, int ul, int sel, double x, double t_mid, int *j, unsigned &probes) {
  const int64_t nl = K.T.nlevels_total;
  const MaMeta mm = K.T.ma_meta[ul];
  int base, cnt;
  if (sel == ARTIS_MA_ACTION_RADDEEXC || sel == ARTIS_MA_ACTION_INTERNALDOWNSAME) {
    base = 0;
    cnt = mm.nd;
  } else if (sel == ARTIS_MA_ACTION_RADRECOMB || sel == ARTIS_MA_ACTION_INTERNALDOWNLOWER) {
    base = mm.nd;
    cnt = mm.nr;
  } else if (sel == ARTIS_MA_ACTION_INTERNALUPSAME) {
    base = mm.nd + mm.nr;
    cnt = mm.nu;
  } else {  // INTERNALUPHIGHER
    base = mm.nd + mm.nr + mm.nu;
    cnt = mm.nt;
  }
  const int mgi = K.C.ne_mgi[k];
  const double ec = K.T.level_epsilon[ul];
  const double *pops = K.C.pops + (int64_t)k * nl;
  const double *corr = K.C.corrphot + (int64_t)k * K.T.ntargets_total;
  auto pop = [&](int u) { return pops[u]; };
  auto cph = [&](int s) { return corr[s]; };
  const int lane = (int)__lane_id();
  auto term_at = [&](int c0) {  // this lane's term of entries [c0, c0 + 64), 0 past the list
    double term = 0.;
    if (c0 + lane < cnt) {
      const MaItem it = ma_rate_at(K, mgi, ul, t_mid, base + c0 + lane, pop, cph);
      switch (sel) {  // the summand of ma_accumulate for this action
        case ARTIS_MA_ACTION_RADDEEXC:
        case ARTIS_MA_ACTION_RADRECOMB: term = it.R * it.et; break;
        case ARTIS_MA_ACTION_INTERNALDOWNSAME:
        case ARTIS_MA_ACTION_INTERNALDOWNLOWER: term = (it.R + it.C) * it.eg; break;
        case ARTIS_MA_ACTION_INTERNALUPSAME: term = (it.R + it.C + 0.) * ec; break;
        default: term = (it.R + it.C) * ec; break;
      }
    }
    return term;
  };
  // Fast path: a wave prefix sum (six shuffle steps, its own rounding) finds the first entry whose running sum
  // exceeds x.  All terms are >= 0, so the reference's sequential sums and the prefix sums both lie within
  // (c0 + 70) u of the exact sums relative to the largest partial sum; when x is farther than twice that from
  // the two sums around the crossing, the sequential scan crosses at the same entry.  Otherwise (or when no sum
  // crosses), the exact path below adds the terms one at a time in list order.
  double base_sum = 0.;
  for (int c0 = 0; c0 < cnt; c0 += 64) {
    double incl = term_at(c0);
    for (int off = 1; off < 64; off <<= 1) {
      const double t = __shfl_up(incl, off, 64);
      if (lane >= off) incl += t;
    }
    incl += base_sum;
    const unsigned long long cross = __ballot(c0 + lane < cnt && incl > x);
    if (cross) {
      const int f = __ffsll((long long)cross) - 1;
      const double s_f = readlane_d(incl, f);
      const double s_prev = f > 0 ? readlane_d(incl, f - 1) : base_sum;
      const double tol = 2.0 * (double)(c0 + 70) * 1.1102230246251565e-16 * s_f;
      if (s_f - x > tol && x - s_prev > tol) {
        probes += (unsigned)(c0 + f + 1);
        *j = c0 + f;
        return sel;
      }
      break;
    }
    base_sum = readlane_d(incl, min(63, cnt - c0 - 1));
  }
  // exact path: the reference's sequential running sum, one term per step from the evaluating lane's register
  double run = 0.;
  for (int c0 = 0; c0 < cnt; c0 += 64) {
    const double term = term_at(c0);
    const int n64 = min(64, cnt - c0);
#pragma unroll 1
    for (int q = 0; q < n64; q++) {
      run += readlane_d(term, q);
      if (run > x) {
        probes += (unsigned)(c0 + q + 1);
        *j = c0 + q;
        return sel;
      }
    }
  }
  probes += (unsigned)cnt;
  return MA_COOP_NOSEL;
}
// the lane's side of that jump: its RNG draws (the action draw, then the transition's or the NT ion's), the jump
// count and histogram, and the selection applied as in the cached step
DEVFN int ma_coop_apply(const Ctx &K, const MaHot &H, const LocalCounters &L, artis_rng &rng, MaLaneR &m, MaEnd &end,
                        int number, int sel, int j, unsigned probes, const MaMetaW &meta) {
  m.n0 = rng.n;
  rng.n++;
  m.ntrans += probes;
  if (sel == MA_COOP_RANDOM) {
    fail(K, ERR_MA_RANDOM, number, m.ul);
    return MA_FAILED;
  }
  if (sel == MA_COOP_NOSEL) {
    fail(K, ERR_MA_SELECT, number, 20);
    return MA_FAILED;
  }
  m.jumps++;
  // (counted exactly, not sampled like the cached jumps: see DevCells::ma_lhist)
  if (H.ma_lhist) atomicAdd(&H.ma_lhist[(int64_t)m.k * H.nlevels_total + m.ul], 1u);
  if (sel == ARTIS_MA_ACTION_COLDEEXC || sel == ARTIS_MA_ACTION_COLRECOMB) {
    end.code = (sel == ARTIS_MA_ACTION_COLDEEXC) ? MA_END_COLDEEXC : MA_END_COLRECOMB;
    end.ion = end.a = end.b = 0;
    return end.code;
  }
  if (sel == ARTIS_MA_ACTION_INTERNALUPHIGHERNT) return ma_apply_nt(K, L, rng, m, number);
  rng.n++;
  return ma_apply_selection(K, H, L, m, end, sel, j, meta.w0.y, meta.w0.z, meta.w0.w);
}

#ifndef ARTIS_MA_SEARCH4
#define ARTIS_MA_SEARCH4 0
#endif
// where a step reads record keys (high halves): k_ma's staged line, or the whole record in global memory
template <bool HI_ONLY>
struct KeysLds {
  lds_uint4 *line;
  int pl;
  DEVFN bool hi_only(const Ctx &) const { return HI_ONLY; }  // (level mode, the COOP instance of k_ma)
  DEVFN bool has(int p) const { return (p >> 6) == pl; }
  DEVFN uint32_t hi(int p) const { return (uint32_t)((lds_u16 *)(line + ((p & 63) >> 3) * 64))[p & 7]; }
  // the 9 action keys (line 0): positions 0-7 packed two per word (one 16-byte LDS read), position 8
  DEVFN void first9(u32x4 &k07, uint32_t &k8) const {
    k07 = line[0];
    k8 = (uint32_t)((lds_u16 *)(line + 64))[0];
  }
};
struct KeysGlobal {
  const uint16_t *rec;
  DEVFN bool hi_only(const Ctx &K) const { return K.C.ma_hi_only != 0; }
  DEVFN bool has(int) const { return true; }
  DEVFN uint32_t hi(int p) const { return (uint32_t)gload(rec + p); }
  DEVFN void first9(u32x4 &k07, uint32_t &k8) const {
    k07 = *(glb_uint4 *)rec;
    k8 = hi(8);
  }
};

// Counts of the 9 action keys (16-bit high halves, non-decreasing) below qh and below qh + 2, in packed 16-bit
// arithmetic: per word of two keys a saturating subtraction from the threshold (non-zero iff key < threshold), a
// min with 1 and a packed add -- no per-key compare / carry chains (each a VCC write the next VALU instruction must
// wait for on gfx950).  nund = keys equal to qh or qh + 1 (undecided at 16 bits).
// (written as VOP3P instructions: from the equivalent C the compiler makes two compares, two selects and a permute
// per word)
DEVFN uint32_t pk_below(uint32_t tt, uint32_t k, uint32_t one) {  // per 16-bit half: k < t ? 1 : 0
  uint32_t d, r;
  asm("v_pk_sub_u16 %0, %1, %2 clamp" : "=v"(d) : "v"(tt), "v"(k));
  asm("v_pk_min_u16 %0, %1, %2" : "=v"(r) : "v"(d), "v"(one));
  return r;
}
DEVFN uint32_t ma_count_below(const u32x4 &k07, uint32_t k8, uint32_t t) {
  // t <= 0xffff: the count of keys < t
  const uint32_t tt = t | (t << 16), one = 0x00010001u;
  const uint32_t a = pk_below(tt, k07.x, one) + pk_below(tt, k07.y, one) + pk_below(tt, k07.z, one) +
                     pk_below(tt, k07.w, one);  // (halves <= 4: no carry between them)
  return (a & 0xffffu) + (a >> 16) + (k8 < t ? 1u : 0u);
}

// meta: the level's MaMetaW (k_ma loads it beside the record-line fetch); z1, z2: the values of the lane's next two
// draws (used only by a step that starts a jump; the RNG counter advances over the draws the jump consumes)
template <class Keys>
DEVFN int ma_step_cached(const Ctx &K, const MaHot &H, const LocalCounters &L, artis_rng &rng, MaLaneR &m, MaEnd &end,
                         int number, const Keys &keys, const MaMetaW &meta, const u32x4 &zw) {
#ifdef ARTIS_STAMPS_SUB  // diagnostic: cycles of the step's sections, added by the first active lane
  struct SubStamp {
    const LocalCounters &L;
    unsigned long long t0, t1 = 0, t2 = 0;
    DEVFN ~SubStamp() {
      const unsigned long long t3 = __builtin_amdgcn_s_memtime();
      if (L.diag && (int)__lane_id() == __ffsll((long long)__ballot(1)) - 1) {
        if (t1) atomicAdd(&L.diag[40], t1 - t0);
        if (t2) atomicAdd(&L.diag[41], t2 - (t1 ? t1 : t0));
        atomicAdd(&L.diag[42], t3 - (t2 ? t2 : (t1 ? t1 : t0)));
        atomicAdd(&L.diag[43], 1ull);
      }
    }
  } sub{L, __builtin_amdgcn_s_memtime()};
#define SUB_STAMP(f) sub.f = __builtin_amdgcn_s_memtime()
#else
#define SUB_STAMP(f) \
  do {               \
  } while (0)
#endif
  const uint16_t *rec = H.ma_key + (size_t)m.line * 64;
  const int doff = meta.w0.y, uoff = meta.w0.z, base_lower = meta.w0.w;
  const uint32_t wnd = (uint32_t)meta.w0.x, wnr = (uint32_t)meta.w1.x, wl1 = (uint32_t)meta.w1.y,
                 wl2 = (uint32_t)meta.w1.z;
  const int nd = (int)(wnd & 0xffffu), nu = (int)(wnd >> 16), nr = (int)(wnr & 0xffffu), nt = (int)(wnr >> 16);
  // the record layout (engine_dev.h ma_layout, MaWalk): only the fields the step reads
  const int lay_sd = (int)(wl1 & 0xffu), lay_md = (int)((wl1 >> 8) & 0xffu), lay_mu = (int)((wl1 >> 16) & 0xffu),
            lay_nbd = (int)(wl1 >> 24), lay_nbu = (int)(wl2 & 0xffu);
  const int lay_hot = meta.w1.w;
  auto cmp = [&](int p, uint32_t hi, auto q, uint32_t qh) -> int {
    if (hi < qh) return -1;
    if (hi > qh + 1) return 1;
    if (keys.hi_only(K)) return 0;  // level-mode records hold the high halves only: undecided -> exact jump
    return ma_key_cmp((hi << 16) | (uint32_t)gload(rec + lay_hot + p), q());
  };
  if (m.sel < 0) {  // a new jump: the action is the first of the 9 running-sum keys (line 0) above q
    m.n0 = rng.n;
    const auto q = [&]() { return ma_q_draw(zw.x, zw.y); };
    const uint32_t qh = ma_qh_draw(zw.y);
    rng.n++;
    u32x4 k07;
    uint32_t k8;
    keys.first9(k07, k8);
    const int nless = (int)ma_count_below(k07, k8, qh);
    // (keys < qh + 2; every 16-bit key is when qh + 2 passes 0xffff)
    const int nle1 = (int)ma_count_below(k07, k8, min(qh + 2, 0xffffu));
    const int nund = (qh >= 0xfffeu ? ARTIS_MA_ACTION_COUNT : nle1) - nless;
    int sel = -1;
    if (nund == 0) {  // the keys are non-decreasing: the first nless are decided below q, the next above
      if (nless < ARTIS_MA_ACTION_COUNT) sel = nless;
    } else {
      for (int a = nless; a < ARTIS_MA_ACTION_COUNT; a++) {
        const int c = cmp(a, keys.hi(a), q, qh);
        if (c > 0) {
          sel = a;
          break;
        }
        if (c == 0) break;
      }
    }
    if (sel < 0) return MA_DEFER;
    m.jumps++;
    // level mode: every 16th jump of a walk credits its (cell, level) pair for the next record placement
    if (H.ma_lhist && (m.jumps & 15u) == 0u) atomicAdd(&H.ma_lhist[(int64_t)m.k * H.nlevels_total + m.ul], 16u);
    if (sel == ARTIS_MA_ACTION_COLDEEXC || sel == ARTIS_MA_ACTION_COLRECOMB) {
      end.code = (sel == ARTIS_MA_ACTION_COLDEEXC) ? MA_END_COLDEEXC : MA_END_COLRECOMB;
      end.ion = end.a = end.b = 0;
      return end.code;
    }
    if (sel == ARTIS_MA_ACTION_INTERNALUPHIGHERNT) return ma_apply_nt(K, L, rng, m, number);
    m.q2lo = zw.z;
    m.q2hi = zw.w;
    m.q2h = ma_qh_draw(zw.w);
    rng.n++;
    m.sel = sel;
    MA_DIAG(sel);
    m.lo = 0;
    m.blk = -1;
    if (sel == ARTIS_MA_ACTION_INTERNALDOWNSAME || sel == ARTIS_MA_ACTION_INTERNALUPSAME) {
      const bool down = sel == ARTIS_MA_ACTION_INTERNALDOWNSAME;
      m.base = down ? 9 : 9 + lay_sd;
      m.end = (int)((wl2 >> (down ? 8 : 16)) & 0xffu);  // separators and suffix, or the array
    } else {
      const int sorted0 = 64 * (1 + lay_nbd + lay_nbu);
      m.base = sorted0 + ((sel == ARTIS_MA_ACTION_RADDEEXC)            ? 0
                          : (sel == ARTIS_MA_ACTION_RADRECOMB)         ? nd
                          : (sel == ARTIS_MA_ACTION_INTERNALDOWNLOWER) ? nd + nr
                                                                       : nd + 2 * nr);  // INTERNALUPHIGHER
      m.end = (sel == ARTIS_MA_ACTION_RADDEEXC) ? nd : (sel == ARTIS_MA_ACTION_INTERNALUPHIGHER) ? nt : nr;
    }
    m.hi = m.end;
  }
  SUB_STAMP(t1);
  // binary search for the first entry above q2, resumed where it stopped.  The inner loop is the branch-light
  // common case (probe on the staged line, decided by the high half); it leaves for a probe off the line
  // (MA_PENDING) or a high half that needs its low half (rare).
  int lo = m.lo, hi = m.hi;
  const int base = m.base;
  const uint32_t q2h = m.q2h;
  unsigned probes = 0;
#if ARTIS_MA_SEARCH4
  // 4-ary steps (three probes per LDS round trip) while the range lies on the staged line, is 4 entries or longer
  // and its probes are decided by their high halves; the binary loop below finishes (the same entry: every
  // narrowing is an exact comparison of sorted keys)
  while (hi - lo >= 4 && keys.has(base + lo) && keys.has(base + hi - 1)) {
    const int len = hi - lo;
    const int m1 = lo + (len >> 2), m2 = lo + (len >> 1), m3 = lo + ((3 * len) >> 2);
    const uint32_t h1 = keys.hi(base + m1), h2 = keys.hi(base + m2), h3 = keys.hi(base + m3);
    if ((h1 - q2h) <= 1u || (h2 - q2h) <= 1u || (h3 - q2h) <= 1u) break;
    probes += 3;
    if (h1 > q2h) {
      hi = m1;
    } else if (h2 > q2h) {
      lo = m1 + 1;
      hi = m2;
    } else if (h3 > q2h) {
      lo = m2 + 1;
      hi = m3;
    } else {
      lo = m3 + 1;
    }
  }
#endif
  while (true) {
    int mid = 0, p = 0;
    uint32_t h = 0;
    while (lo < hi) {
      mid = (lo + hi) >> 1;
      p = base + mid;
      if (!keys.has(p)) break;
      h = keys.hi(p);
      if ((h - q2h) <= 1u) break;  // high half qh or qh + 1: undecided at 16 bits
      probes++;
      if (h > q2h)
        hi = mid;
      else
        lo = mid + 1;
    }
    if (lo >= hi) break;
    if (!keys.has(p)) {
      m.lo = lo;
      m.hi = hi;
      m.pline = p >> 6;
      m.ntrans += probes;
      MA_DIAG(16 + m.sel);
      return MA_PENDING;
    }
    probes++;
    const int c = keys.hi_only(K) ? 0 : ma_key_cmp((h << 16) | (uint32_t)gload(rec + lay_hot + p), ma_q_draw(m.q2lo, m.q2hi));
    if (c == 0) {
      m.ntrans += probes;
      m.jumps--;
      m.sel = -1;
      m.pline = 0;
      return MA_DEFER;
    }
    if (c > 0)
      hi = mid;
    else
      lo = mid + 1;
  }
  m.ntrans += probes;
  SUB_STAMP(t2);
  const int sel = m.sel;
  if (sel == ARTIS_MA_ACTION_INTERNALDOWNSAME || sel == ARTIS_MA_ACTION_INTERNALUPSAME) {
    const bool down = sel == ARTIS_MA_ACTION_INTERNALDOWNSAME;
    const int cnt = down ? nd : nu, nb = down ? lay_nbd : lay_nbu, suf = down ? lay_md : lay_mu;
    // separators and suffix searched: the key is in block lo (round-4 layout: the last if no separator is above
    // q2), or suffix entry lo - nb
    if (nb && m.blk < 0 && lo < nb) {
      m.blk = lo;
      m.base = 64 * (1 + (down ? 0 : lay_nbd) + lo);
      m.lo = 0;
      m.end = m.hi = min(64, cnt - suf - 64 * lo);
      m.pline = m.base >> 6;
      MA_DIAG(16 + sel);
      return MA_PENDING;
    }
    const int j = !nb ? lo : (m.blk >= 0) ? 64 * m.blk + lo : cnt - suf + (lo - nb);
    const bool found = lo < m.end;
#ifdef ARTIS_STAMPS
    // where the up-same selections of blocked arrays fall: [9] count, [10] in the line-0 suffix, [11] the first
    // 16, [12] the last 16, [13] the first `suffix` entries, [14] the sum of the array sizes, [15] the sum of the
    // suffix sizes, [25 + q] quarter q of the array
    if (!down && nb && L.diag && found) {
      MA_DIAG(9);
      if (j >= cnt - suf) MA_DIAG(10);
      if (j < 16) MA_DIAG(11);
      if (j >= cnt - 16) MA_DIAG(12);
      if (j < suf) MA_DIAG(13);
      atomicAdd(&L.diag[14], (unsigned long long)cnt);
      atomicAdd(&L.diag[15], (unsigned long long)suf);
      MA_DIAG(25 + min(3, 4 * j / cnt));
    }
#endif
    m.sel = -1;
    m.pline = 0;
    if (!found) {
      fail(K, ERR_MA_SELECT, number, 10 + sel);
      return MA_FAILED;
    }
    typedef const __attribute__((address_space(1))) uint64_t glb_u64;
    const uint64_t tw = *(glb_u64 *)(down ? H.down_target + doff + j : H.up_target + uoff + j);
    m.ul = (int)(uint32_t)tw;
    m.line = ma_line(H, m.rowline, m.k, m.ul, (int)(uint32_t)(tw >> 32));
    return MA_CONTINUE;
  }
  const bool found = lo < m.end;
  m.sel = -1;
  m.pline = 0;
  if (!found) {
    fail(K, ERR_MA_SELECT, number, 10 + sel);
    return MA_FAILED;
  }
  return ma_apply_selection(K, H, L, m, end, sel, lo, doff, uoff, base_lower);
}

// One whole jump of the cached walk from the record in global memory (the megakernel's do_macroatom): the step
// never waits for a line, so it runs to the end of the jump (the block of a two-level array: a second call).
DEVFN int ma_jump_cached_global(const Ctx &K, const LocalCounters &L, artis_rng &rng, MaLaneC &mc, MaEnd &end,
                                int number) {
  u32x4 zw;
  artis_rng_jump_words(&rng, (uint32_t *)&zw);
  MaLaneR m;
  static_cast<MaLaneC &>(m) = mc;
  m.sel = -1;
  m.pline = 0;
  const MaMetaW meta = ma_walk_load(K, m.ul);
  const KeysGlobal keys{K.C.ma_key + (size_t)m.line * 64};
  int r;
  do {
    r = ma_step_cached(K, ma_hot(K), L, rng, m, end, number, keys, meta, zw);
  } while (r == MA_PENDING);
  if (r == MA_DEFER) rng.n = m.n0;
  mc = static_cast<MaLaneC &>(m);
  return r;
}


// the fb deactivation (macroatom.cc:340-380): select_continuum_nu's quadrature, noinline (run on copies, cold_call)
DEVNI void ma_finish_fb(Tx &x, Pkt &p, const MaEnd &e, double fb_nu) {
  const Ctx &K = x.K;
  const int element = p.ma_element;
  const int uiu = K.T.level_ui[e.b];
  const int ion = uiu - K.T.elem_uniqueionoffset[element] - 1, lower = e.a;
  const int upperionlevel = e.b - K.T.ion_uniqueleveloffset[uiu];
  const float T_e = K.C.Te[cell_mgi(K, p.where)];
  p.nu_cmf = fb_nu >= 0. ? fb_nu : select_continuum_nu(x, element, ion, lower, upperionlevel, T_e);
  lctr(x.L, CTR_MA_STAT_DEACTIVATION_FB);
  p.last_event = 2;
  emitt_rpkt(x, p);
  p.next_trans = 0;
  {  // get_continuumindex (atomic.cc:16-30)
    int target = 0;
    for (int t = 0; t < get_nphixstargets(K, element, ion, lower); t++)
      if (get_phixsupperlevel(K, element, ion, lower, t) == upperionlevel) {
        target = t;
        break;
      }
    p.emissiontype = K.T.level_cont_index[ulev(K, element, ion, lower)] - target;
  }
  p.em_pos[0] = p.pos[0];
  p.em_pos[1] = p.pos[1];
  p.em_pos[2] = p.pos[2];
  p.em_time = (int)p.prop_time;
  p.nscatterings = 0;
  if (K.V.on) vpkt_spawn(x, p, 3);  // macroatom.cc:376-379
}

// the deactivation branches of do_macroatom (macroatom.cc:222-380, 445-462) and its trailer (macroatom.cc:475-482);
// `jumps` passes of the loop each added one interaction.  Inline (bb and collisional in the caller's registers);
// ma_finish is the noinline form for the kernels that run it on a copy.
DEVFN void ma_finish_inl(Tx &x, Pkt &p, const MaEnd &e, unsigned jumps, double fb_nu = -1.) {
  const Ctx &K = x.K;
  const int element = p.ma_element;
  p.interactions += (int)jumps;
  if (e.code == MA_END_BB) {
    const int linelistindex = e.a >= 0 ? e.a : K.T.downtrans_lineindex[-1 - e.a], ul = e.b;
    const int ion = K.T.level_ui[ul] - K.T.elem_uniqueionoffset[element];
    if (K.R.record_linestat) atomicAdd(&K.E.ecounter[linelistindex], 1);
    const int lower = K.T.line_lower[linelistindex];
    const double epsilon_trans = K.T.level_epsilon[ul] - epsilon(K, element, ion, lower);
    double oldnucmf = 0.;
    if (p.last_event == 1) oldnucmf = p.nu_cmf;
    p.nu_cmf = epsilon_trans / ARTIS_H;
    if (p.last_event == 1) lctr(x.L, (oldnucmf < p.nu_cmf) ? CTR_UPSCATTER : CTR_DOWNSCATTER);
    lctr(x.L, CTR_MA_STAT_DEACTIVATION_BB);
    p.last_event = 0;
    emitt_rpkt(x, p);
    if (linelistindex == p.ma_activatingline) lctr(x.L, CTR_RESONANCESCATTERINGS);
    p.next_trans = linelistindex + 1;
    p.emissiontype = linelistindex;
    p.em_pos[0] = p.pos[0];
    p.em_pos[1] = p.pos[1];
    p.em_pos[2] = p.pos[2];
    p.em_time = (int)p.prop_time;
    p.nscatterings = 0;
    if (K.V.on) vpkt_spawn(x, p, 3);  // macroatom.cc:292-295
  } else if (e.code == MA_END_COLDEEXC || e.code == MA_END_COLRECOMB) {
    const bool deexc = e.code == MA_END_COLDEEXC;
    lctr(x.L, deexc ? CTR_MA_STAT_DEACTIVATION_COLLDEEXC : CTR_MA_STAT_DEACTIVATION_COLLRECOMB);
    p.last_event = deexc ? 10 : 11;
    p.type = ARTIS_TYPE_KPKT;
    safeadd(&K.E.colheat[cell_mgi(K, p.where)], p.e_cmf);
  } else if (e.code == MA_END_FB) {
    cold_call(x, p, [&](Tx &tx, Pkt &tp) { ma_finish_fb(tx, tp, e, fb_nu); });
  }
  if (p.trueemissiontype < 0) {
    p.trueemissiontype = p.emissiontype;
    p.trueemissionvelocity = (float)(vec_len(p.em_pos) / p.em_time);
    p.trueem_time = p.em_time;
  }
}
DEVNI void ma_finish(Tx &x, Pkt &p, const MaEnd &e, unsigned jumps) { ma_finish_inl(x, p, e, jumps); }

#define MA_MAX_JUMPS 10000000u

// macroatom.cc:416-482 (megakernel form: walk + finish)
DEVNI void do_macroatom(Tx &x, Pkt &p) {
  const Ctx &K = x.K;
  const int mgi = cell_mgi(K, p.where);
  if (K.C.thick[mgi] == 1) {
    x.err(ERR_THICK_MA, p.number, mgi);
    return;
  }
  MaEnd e;
  e.code = MA_CONTINUE;
  int r;
  unsigned jumps;
  unsigned long long ntrans;
  {
    // the walk over the key records where the cell has them (row mode, or a (cell, level) record of level mode);
    // a jump without a record or with an undecided key comparison is made with the exact sums (ma_jump_exact)
    MaLaneC m;
    m.k = K.C.ne_index[mgi];
    m.rowline = ma_rowline(K, m.k);
    ma_set_level(K, m, ulev(K, p.ma_element, p.ma_ion, p.ma_level));
    m.jumps = 0;
    m.ntrans = 0;
    const double t_mid = K.G.ts_mid[x.nts];
    while (true) {
      const uint32_t n0 = x.rng.n;
      r = (m.line == MA_NOLINE) ? MA_DEFER : ma_jump_cached_global(K, x.L, x.rng, m, e, p.number);
      if (r == MA_DEFER) {
        x.rng.n = n0;
        r = ma_jump_exact(K, x.L, x.rng, m, e, p.number, t_mid);
      }
      if (r != MA_CONTINUE || m.jumps >= MA_MAX_JUMPS) break;
    }
    jumps = m.jumps;
    ntrans = m.ntrans;
  }
  if (r == MA_CONTINUE) {
    x.err(ERR_STUCK, p.number, 2);
    return;
  }
  lwork(x.L, WK_MA_JUMPS, jumps);
  lwork(x.L, WK_MA_TRANS, ntrans);
  if (r == MA_FAILED) {
    x.ok = false;
    return;
  }
  ma_finish(x, p, e, jumps);
}

// ------------------------------------------------------------------------------------------ k-packets
// kpkt.cc:428-446
DEVFN double sample_planck(Tx &x, double T, int number) {
  const double nu_peak = 5.879e10 * T;
  const double B_peak = dbb(nu_peak, T, 1);
  for (int tries = 0; tries < 10000000; tries++) {
    const double zrand = artis_rng_uniform(&x.rng);
    const double zrand2 = artis_rng_uniform(&x.rng);
    const double nu = x.K.G.nu_min_r + zrand * (x.K.G.nu_max_r - x.K.G.nu_min_r);
    if (zrand2 * B_peak <= dbb(nu, T, 1)) return nu;
  }
  x.err(ERR_STUCK, number, 3);
  return x.K.G.nu_min_r;
}
// kpkt.cc:448-475
DEVNI void do_kpkt_bb(Tx &x, Pkt &p) {
  const int mgi = cell_mgi(x.K, p.where);
  const float T_e = x.K.C.Te[mgi];
  p.nu_cmf = sample_planck(x, T_e, p.number);
  emitt_rpkt(x, p);
  p.next_trans = 0;
  lctr(x.L, CTR_K_STAT_TO_R_BB);
  p.interactions++;
  p.last_event = 6;
  p.emissiontype = -9999999;
  p.em_pos[0] = p.pos[0];
  p.em_pos[1] = p.pos[1];
  p.em_pos[2] = p.pos[2];
  p.em_time = (int)p.prop_time;
  p.nscatterings = 0;
}
// kpkt.cc:477-797 (cumulative cooling list from the per-cell table)
// an fb emission whose frequency the wave computes (wave_select_continuum_nu): the continuum and the draw
struct FbReq {
  bool want = false;
  int e = 0, ion = 0, lower = 0, upper = 0;
  float T_e = 0.f;
  double zrand = 0.;
};

// kpkt.cc:661-700, the fb cooling branch after the frequency
DEVFN void kpkt_fb_tail(Tx &x, Pkt &p, int el, int lowerion, int level, int upper, double nu) {
  const Ctx &K = x.K;
  p.nu_cmf = nu;
  emitt_rpkt(x, p);
  p.next_trans = 0;
  lctr(x.L, CTR_K_STAT_TO_R_FB);
  p.interactions += 1;
  p.last_event = 7;
  int target = 0;
  for (int t = 0; t < get_nphixstargets(K, el, lowerion, level); t++)
    if (get_phixsupperlevel(K, el, lowerion, level, t) == upper) {
      target = t;
      break;
    }
  p.emissiontype = K.T.level_cont_index[ulev(K, el, lowerion, level)] - target;
  p.trueemissiontype = p.emissiontype;
  p.em_pos[0] = p.pos[0];
  p.em_pos[1] = p.pos[1];
  p.em_pos[2] = p.pos[2];
  p.em_time = (int)p.prop_time;
  p.nscatterings = 0;
  if (K.V.on) vpkt_spawn(x, p, 2);  // kpkt.cc:691-694
}

// kpkt.cc:477-797.  fb: nullptr -- the fb frequency is computed here (select_continuum_nu); otherwise an fb channel
// stops after its draw with the request in *fb (the caller's wave computes the frequency, then kpkt_fb_tail)
DEVNI void do_kpkt(Tx &x, Pkt &p, double t2, FbReq *fb = nullptr) {
  const Ctx &K = x.K;
  const double t1 = p.prop_time;
  const int mgi = cell_mgi(K, p.where);
  const int k = K.C.ne_index[mgi];
  const float T_e = K.C.Te[mgi];
  lwork(x.L, WK_KPKT, 1);
  double deltat = 0.;
  if (x.nts < K.R.n_kpktdiffusion_timesteps) deltat = K.R.kpktdiffusion_timescale * K.G.ts_width[x.nts];
  const double t_current = t1 + deltat;
  if (!(t_current <= t2)) {
    const double s = t2 / t1;
    p.pos[0] *= s;
    p.pos[1] *= s;
    p.pos[2] *= s;
    p.prop_time = t2;
    return;
  }
  {
    const double s = t_current / t1;
    p.pos[0] *= s;
    p.pos[1] *= s;
    p.pos[2] *= s;
  }
  p.prop_time = t_current;
  double coolingsum = 0.;
  const double zrand = artis_rng_uniform(&x.rng);
  const double rndcool = zrand * K.C.totalcooling[mgi];
  double oldcoolingsum = 0.;
  int element = -1, ion = -1;
  for (element = 0; element < K.T.nelements; element++) {
    const int nions = get_nions(K, element);
    for (ion = 0; ion < nions; ion++) {
      oldcoolingsum = coolingsum;
      coolingsum += K.C.cooling_contrib_ion[(int64_t)mgi * K.T.nions_total + uion(K, element, ion)];
      if (coolingsum > rndcool) break;
    }
    if (coolingsum > rndcool) break;
  }
  if (element >= K.T.nelements || ion >= get_nions(K, element)) {
    x.err(ERR_KPKT, p.number, 0);
    return;
  }
  const int ui = uion(K, element, ion);
  const int ilow = K.T.ion_coolingoffset[ui];
  const int ihigh = ilow + K.T.ion_ncoolingterms[ui] - 1;
  const double *cc = K.C.cooling + (int64_t)k * K.T.ncoolingterms;
  int lo = ilow, hi = ihigh + 1;
  while (lo < hi) {
    const int mid = lo + (hi - lo) / 2;
    if (cc[mid] < rndcool)
      lo = mid + 1;
    else
      hi = mid;
  }
  int icool = lo;
  if (icool > ihigh) icool = ihigh;  // deviation D6
  lwork(x.L, WK_KPKT_TERMS, (unsigned long long)(icool - ilow + 1));
  const int ctype = K.T.cool_type[icool];
  if (ctype == ARTIS_COOLINGTYPE_FF) {
    const double zr = artis_rng_uniform_pos(&x.rng);
    p.nu_cmf = -ARTIS_KB * T_e / ARTIS_H * log(zr);
    emitt_rpkt(x, p);
    p.next_trans = 0;
    lctr(x.L, CTR_K_STAT_TO_R_FF);
    p.interactions += 1;
    p.last_event = 6;
    p.emissiontype = -9999999;
    p.em_pos[0] = p.pos[0];
    p.em_pos[1] = p.pos[1];
    p.em_pos[2] = p.pos[2];
    p.em_time = (int)p.prop_time;
    p.nscatterings = 0;
    if (K.V.on) vpkt_spawn(x, p, 2);  // kpkt.cc:631-634
  } else if (ctype == ARTIS_COOLINGTYPE_FB) {
    const int el = K.T.cool_element[icool];
    const int lowerion = K.T.cool_ion[icool];
    const int level = K.T.cool_level[icool];
    const int upper = K.T.cool_upper[icool];
    if (fb) {
      fb->want = true;
      fb->e = el;
      fb->ion = lowerion;
      fb->lower = level;
      fb->upper = upper;
      fb->T_e = T_e;
      fb->zrand = 1. - artis_rng_uniform(&x.rng);  // select_continuum_nu's draw
      return;
    }
    kpkt_fb_tail(x, p, el, lowerion, level, upper, select_continuum_nu(x, el, lowerion, level, upper, T_e));
  } else if (ctype == ARTIS_COOLINGTYPE_COLLEXC) {
    const float nne = K.C.nne[mgi];
    const double contrib_low = (icool > ilow) ? cc[icool - 1] : oldcoolingsum;
    double contrib = contrib_low;
    const int level = K.T.cool_level[icool];
    const int ul = ulev(K, element, ion, level);
    const double nnlevel = K.C.pops[(int64_t)k * K.T.nlevels_total + ul];
    const double statweight = stat_weight(K, element, ion, level);
    int upper = -1;
    const int nuptrans = K.T.level_nuptrans[ul];
    const int uoff = K.T.level_uptrans_offset[ul];
    // the running sum over the level's up-transitions (kpkt.cc:660-700) from the packed excitation items: one
    // independent 32-byte load per line, four in flight (the line index -> upper level -> its epsilon and statistical
    // weight chain of three dependent loads per line made this loop the k-packet's cost on large atoms); the upper level
    // of the selected line only is looked up
    const TeExcItem *items = K.T.exc_items + uoff;
    int sel = -1;
    for (int i0 = 0; i0 < nuptrans && sel < 0; i0 += 4) {
      TeExcItem it[4];
#pragma unroll
      for (int q = 0; q < 4; q++) it[q] = items[min(i0 + q, nuptrans - 1)];
#pragma unroll
      for (int q = 0; q < 4; q++) {
        if (i0 + q >= nuptrans || sel >= 0) break;
        contrib += nnlevel * te_col_exc(it[q], T_e, nne, statweight) * it[q].epsilon_trans;
        if (contrib >= rndcool) sel = i0 + q;
      }
    }
    if (sel < 0 && nuptrans > 0) sel = nuptrans - 1;  // D6
    if (sel >= 0) upper = K.T.line_upper[K.T.uptrans_lineindex[uoff + sel]];
    if (upper < 0) {
      x.err(ERR_KPKT, p.number, 1);
      return;
    }
    p.ma_element = element;
    p.ma_ion = ion;
    p.ma_level = upper;
    p.ma_activatingline = -99;
    p.type = ARTIS_TYPE_MA;
    lctr(x.L, CTR_MA_STAT_ACTIVATION_COLLEXC);
    lctr(x.L, CTR_K_STAT_TO_MA_COLLEXC);
    p.interactions += 1;
    p.last_event = 8;
    p.trueemissiontype = -1;
    p.trueemissionvelocity = -1;
  } else if (ctype == ARTIS_COOLINGTYPE_COLLION) {
    p.ma_element = K.T.cool_element[icool];
    p.ma_ion = K.T.cool_ion[icool] + 1;
    p.ma_level = K.T.cool_upper[icool];
    p.ma_activatingline = -99;
    p.type = ARTIS_TYPE_MA;
    lctr(x.L, CTR_MA_STAT_ACTIVATION_COLLION);
    lctr(x.L, CTR_K_STAT_TO_MA_COLLION);
    p.interactions += 1;
    p.last_event = 9;
    p.trueemissiontype = -1;
    p.trueemissionvelocity = -1;
  } else {
    x.err(ERR_KPKT, p.number, 2);
  }
}

#endif
