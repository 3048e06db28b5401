// qag.h -- NO_LUT_PHOTOION corrected photoionisation coefficients on the GPU: calculate_corrphotoioncoeff_integral
// (ratecoeff.cc:1159-1245) for every (non-empty cell, photoionisation target), one wave per integral.
//
// The reference integrates with gsl_integration_qag(epsabs 0, epsrel 1e-3, GSLWSIZE intervals, GSL_INTEG_GAUSS61).
// This is that algorithm (GSL 2.x integration/qag.c, qk.c, qpsrt.c), with the 61 integrand evaluations of each
// Gauss-Kronrod rule spread over the wave's lanes: lane 0 the centre, lanes 1..30 the left nodes, lanes 31..60
// the right nodes.  The rule's sums, the error estimate and the interval bookkeeping (bisection of the interval
// with the largest error, the error list ordered by qpsrt) then run on every lane alike, in GSL's operation
// order -- the same values on every lane, each lane reading back only what it wrote itself.  The error list and
// its order (walked by qpsrt at every bisection) sit in LDS for the first QAG_LDS intervals, the interval ends,
// results and levels (touched O(1) times per bisection) in a per-wave global workspace of GSLWSIZE entries.
#ifndef ARTIS_QAG_H
#define ARTIS_QAG_H

#include "artis_qk61.h"

#define QAG_LIMIT 16384  // GSLWSIZE (artisoptions_nltenebular.h:75)

struct QagWs {
  double *alist, *blist, *rlist, *elist;  // [nwaves * QAG_LIMIT]
  int32_t *order, *level;
};

__constant__ double c_qk61_xgk[31] = ARTIS_QK61_XGK;
__constant__ double c_qk61_wg[15] = ARTIS_QK61_WG;
__constant__ double c_qk61_wgk[31] = ARTIS_QK61_WGK;

#define QAG_EPS 2.2204460492503131e-16
#define QAG_DMIN 2.2250738585072014e-308

// integration/qk.c rescale_error
DEVFN double qag_rescale_error(double err, const double result_abs, const double result_asc) {
  err = fabs(err);
  if (result_asc != 0 && err != 0) {
    const double scale = pow((200 * err / result_asc), 1.5);
    if (scale < 1)
      err = result_asc * scale;
    else
      err = result_asc;
  }
  if (result_abs > 2 * QAG_DMIN / (50 * QAG_EPS)) {
    const double min_err = 50 * QAG_EPS * result_abs;
    if (min_err > err) err = min_err;
  }
  return err;
}

// integration/qk.c gsl_integration_qk with the 61-point rule; f evaluated once per lane, sums on every lane
template <typename F>
DEVFN void qag_qk61(const F &f, double a, double b, double *s_f, double *result, double *abserr, double *resabs,
                    double *resasc) {
  const int lane = threadIdx.x & 63;
  const double center = 0.5 * (a + b);
  const double half_length = 0.5 * (b - a);
  const double abs_half_length = fabs(half_length);
  if (lane < 61) {
    double x;
    if (lane == 0) {
      x = center;
    } else {
      const int j = (lane <= 30) ? lane - 1 : lane - 31;
      const double abscissa = half_length * c_qk61_xgk[j];
      x = (lane <= 30) ? center - abscissa : center + abscissa;
    }
    s_f[lane] = f(x);
  }
  __syncthreads();
  const double f_center = s_f[0];
  double result_gauss = 0;
  double result_kronrod = f_center * c_qk61_wgk[30];
  double result_abs = fabs(result_kronrod);
  for (int j = 0; j < 15; j++) {
    const int jtw = j * 2 + 1;
    const double fval1 = s_f[1 + jtw], fval2 = s_f[31 + jtw];
    const double fsum = fval1 + fval2;
    result_gauss += c_qk61_wg[j] * fsum;
    result_kronrod += c_qk61_wgk[jtw] * fsum;
    result_abs += c_qk61_wgk[jtw] * (fabs(fval1) + fabs(fval2));
  }
  for (int j = 0; j < 15; j++) {
    const int jtwm1 = j * 2;
    const double fval1 = s_f[1 + jtwm1], fval2 = s_f[31 + jtwm1];
    result_kronrod += c_qk61_wgk[jtwm1] * (fval1 + fval2);
    result_abs += c_qk61_wgk[jtwm1] * (fabs(fval1) + fabs(fval2));
  }
  const double mean = result_kronrod * 0.5;
  double result_asc = c_qk61_wgk[30] * fabs(f_center - mean);
  for (int j = 0; j < 30; j++) result_asc += c_qk61_wgk[j] * (fabs(s_f[1 + j] - mean) + fabs(s_f[31 + j] - mean));
  __syncthreads();  // s_f is reused by the next rule
  const double err = (result_kronrod - result_gauss) * half_length;
  result_kronrod *= half_length;
  result_abs *= abs_half_length;
  result_asc *= abs_half_length;
  *result = result_kronrod;
  *resabs = result_abs;
  *resasc = result_asc;
  *abserr = qag_rescale_error(err, result_abs, result_asc);
}

// The error list and its order (the arrays qpsrt walks, O(size) dependent reads per bisection) live in LDS for the
// first QAG_LDS intervals; intervals beyond that, up to GSLWSIZE, in the wave's global workspace.
#define QAG_LDS 4096
struct QagLists {
  double *s_el;
  int32_t *s_ord;
  double *g_el;
  int32_t *g_ord;
  DEVFN double el(int i) const { return i < QAG_LDS ? s_el[i] : g_el[i]; }
  DEVFN void set_el(int i, double v) const {
    if (i < QAG_LDS)
      s_el[i] = v;
    else
      g_el[i] = v;
  }
  DEVFN int32_t ord(int i) const { return i < QAG_LDS ? s_ord[i] : g_ord[i]; }
  DEVFN void set_ord(int i, int32_t v) const {
    if (i < QAG_LDS)
      s_ord[i] = v;
    else
      g_ord[i] = v;
  }
};

// integration/qpsrt.c on the wave's workspace (ordered list of error indices)
DEVFN void qag_qpsrt(const QagLists &Q, int size, int &nrmax, int &imax) {
  const int last = size - 1;
  const int limit = QAG_LIMIT;
  int i_nrmax = nrmax;
  int i_maxerr = Q.ord(i_nrmax);
  if (last < 2) {
    Q.set_ord(0, 0);
    Q.set_ord(1, 1);
    imax = i_maxerr;
    return;
  }
  const double errmax = Q.el(i_maxerr);
  while (i_nrmax > 0 && errmax > Q.el(Q.ord(i_nrmax - 1))) {
    Q.set_ord(i_nrmax, Q.ord(i_nrmax - 1));
    i_nrmax--;
  }
  const int top = (last < (limit / 2 + 2)) ? last : (limit - last + 1);
  int i = i_nrmax + 1;
  while (i < top && errmax < Q.el(Q.ord(i))) {
    Q.set_ord(i - 1, Q.ord(i));
    i++;
  }
  Q.set_ord(i - 1, i_maxerr);
  const double errmin = Q.el(last);
  int k = top - 1;
  while (k > i - 2 && errmin >= Q.el(Q.ord(k))) {
    Q.set_ord(k + 1, Q.ord(k));
    k--;
  }
  Q.set_ord(k + 1, last);
  imax = Q.ord(i_nrmax);
  nrmax = i_nrmax;
}

// integration/qag.c; returns the GSL status (0, 18 GSL_EROUND, 21 GSL_ESING, 11 GSL_EMAXITER, 5 GSL_EFAILED)
template <typename F>
DEVFN int qag61(const F &f, double a, double b, double epsabs, double epsrel, double *al, double *bl, double *rl,
                const QagLists &Q, int32_t *lev, double *s_f, double *result, double *abserr) {
  const int limit = QAG_LIMIT;
  int size = 0, nrmax = 0, imax = 0;
  al[0] = a;
  bl[0] = b;
  rl[0] = 0.0;
  Q.set_el(0, 0.0);
  Q.set_ord(0, 0);
  lev[0] = 0;
  *result = 0;
  *abserr = 0;
  double result0, abserr0, resabs0, resasc0;
  qag_qk61(f, a, b, s_f, &result0, &abserr0, &resabs0, &resasc0);
  size = 1;
  rl[0] = result0;
  Q.set_el(0, abserr0);
  double tolerance = fmax(epsabs, epsrel * fabs(result0));
  const double round_off = 50 * QAG_EPS * resabs0;
  if (abserr0 <= round_off && abserr0 > tolerance) {
    *result = result0;
    *abserr = abserr0;
    return 18;
  } else if ((abserr0 <= tolerance && abserr0 != resasc0) || abserr0 == 0.0) {
    *result = result0;
    *abserr = abserr0;
    return 0;
  }
  double area = result0;
  double errsum = abserr0;
  int iteration = 1;
  int roundoff_type1 = 0, roundoff_type2 = 0, error_type = 0;
  do {
    const int ii = imax;
    const double a_i = al[ii], b_i = bl[ii], r_i = rl[ii], e_i = Q.el(ii);
    const double a1 = a_i;
    const double b1 = 0.5 * (a_i + b_i);
    const double a2 = b1;
    const double b2 = b_i;
    double area1, area2, error1, error2, resasc1, resasc2, resabs1, resabs2;
    qag_qk61(f, a1, b1, s_f, &area1, &error1, &resabs1, &resasc1);
    qag_qk61(f, a2, b2, s_f, &area2, &error2, &resabs2, &resasc2);
    const double area12 = area1 + area2;
    const double error12 = error1 + error2;
    errsum += (error12 - e_i);
    area += area12 - r_i;
    if (resasc1 != error1 && resasc2 != error2) {
      const double delta = r_i - area12;
      if (fabs(delta) <= 1.0e-5 * fabs(area12) && error12 >= 0.99 * e_i) roundoff_type1++;
      if (iteration >= 10 && error12 > e_i) roundoff_type2++;
    }
    tolerance = fmax(epsabs, epsrel * fabs(area));
    if (errsum > tolerance) {
      if (roundoff_type1 >= 6 || roundoff_type2 >= 20) error_type = 2;
      const double tmp = (1 + 100 * QAG_EPS) * (fabs(a2) + 1000 * QAG_DMIN);
      if (fabs(a1) <= tmp && fabs(b2) <= tmp) error_type = 3;
    }
    // integration/workspace update(): the larger-error half stays at i_max, the other is appended
    const int i_new = size;
    const int new_level = lev[ii] + 1;
    if (error2 > error1) {
      al[ii] = a2;
      rl[ii] = area2;
      Q.set_el(ii, error2);
      lev[ii] = new_level;
      al[i_new] = a1;
      bl[i_new] = b1;
      rl[i_new] = area1;
      Q.set_el(i_new, error1);
      lev[i_new] = new_level;
    } else {
      bl[ii] = b1;
      rl[ii] = area1;
      Q.set_el(ii, error1);
      lev[ii] = new_level;
      al[i_new] = a2;
      bl[i_new] = b2;
      rl[i_new] = area2;
      Q.set_el(i_new, error2);
      lev[i_new] = new_level;
    }
    size++;
    qag_qpsrt(Q, size, nrmax, imax);
    iteration++;
  } while (iteration < limit && !error_type && errsum > tolerance);
  double result_sum = 0;
  for (int k = 0; k < size; k++) result_sum += rl[k];
  *result = result_sum;
  *abserr = errsum;
  if (errsum <= tolerance) return 0;
  if (error_type == 2) return 18;
  if (error_type == 3) return 21;
  if (iteration == limit) return 11;
  return 5;
}

// ratecoeff.cc:1255-1261: DETAILED_BF_ESTIMATORS_ON from DETAILED_BF_ESTIMATORS_USEFROMTIMESTEP, the previous
// timestep's normalised bf-rate estimator of the target's continuum replaces the coefficient when positive
DEVFN bool bfrate_override(const Ctx &K, int mgi, int slot) {
  if (!(K.R.detailed_bf && K.R.nts >= K.R.detailed_bf_usefrom)) return false;
  const int ic = K.T.slot_allcont[slot];
  return ic >= 0 && (double)K.C.bfrate_est[(int64_t)mgi * K.T.nbf + ic] > 0;
}

// ratecoeff.cc:1184-1245 calculate_corrphotoioncoeff_integral for every (cell, target) the estimator does not
// cover; blocks of one wave, grid-strided over n_nonempty * ntargets items
__global__ __launch_bounds__(64) void k_corrphot_integral(Ctx K, const int32_t *target_ul, const int32_t *target_t,
                                                          QagWs ws) {
  __shared__ double s_f[64];
  __shared__ double s_el[QAG_LDS];
  __shared__ int32_t s_ord[QAG_LDS];
  const int64_t ntg = K.T.ntargets_total;
  const int64_t total = (int64_t)K.C.n_nonempty * ntg;
  const int64_t wbase = (int64_t)blockIdx.x * QAG_LIMIT;
  double *al = ws.alist + wbase, *bl = ws.blist + wbase, *rl = ws.rlist + wbase;
  int32_t *lev = ws.level + wbase;
  const QagLists Q{s_el, s_ord, ws.elist + wbase, ws.order + wbase};
  for (int64_t item = blockIdx.x; item < total; item += gridDim.x) {
    const int k = (int)(item / ntg);
    const int slot = (int)(item % ntg);
    const int mgi = K.C.ne_mgi[k];
    if (bfrate_override(K, mgi, slot)) continue;
    const int ul = target_ul[slot];
    const int t = target_t[slot];
    const int ui = K.T.level_ui[ul];
    const int e = K.T.ion_element[ui];
    const int i = ui - K.T.elem_uniqueionoffset[e];
    const int l = ul - K.T.ion_uniqueleveloffset[ui];
    const double *pops = K.C.pops + (int64_t)k * K.T.nlevels_total;
    const double E_threshold = get_phixs_threshold(K, e, i, l, t);
    const double nu_threshold = ARTIS_ONEOVERH * E_threshold;
    const double nu_max_phixs = nu_threshold * K.T.last_phixs_nuovernuedge;
    const float T_e = K.C.Te[mgi];
    const double nnlevel = pops[ul];
    const double nne = K.C.nne[mgi];
    const int upperionlevel = get_phixsupperlevel(K, e, i, l, t);
    const double sf = calculate_sahafact(K, e, i, l, upperionlevel, T_e, ARTIS_H * nu_threshold);
    const double nnupperionlevel = pops[ulev(K, e, i + 1, upperionlevel)];
    double departure_ratio = nnlevel > 0. ? nnupperionlevel / nnlevel * nne * sf : 1.0;
    if (!isfinite(departure_ratio)) departure_ratio = 0.;
    const float *xs = level_photoion_xs(K, e, i, l);
    // integrand_corrphotoioncoeff_custom_radfield (ratecoeff.cc:1159-1181)
    auto integrand = [&](double nu) {
      double corrfactor = 1. - departure_ratio * exp(-ARTIS_HOVERKB * nu / T_e);
      if (corrfactor < 0) corrfactor = 0.;
      const float sigma_bf = (float)photoionization_crosssection_fromtable(K, xs, nu_threshold, nu);
      const double Jnu = radfield_J(K, mgi, nu);
      return ARTIS_ONEOVERH * sigma_bf / nu * Jnu * corrfactor;
    };
    double gammacorr = 0., error = 0.;
    const int status = qag61(integrand, nu_threshold, nu_max_phixs, 0., 1e-3, al, bl, rl, Q, lev, s_f, &gammacorr,
                             &error);
    if (status != 0 && (status != 18 || (error / gammacorr) > 1e-1)) {
      if (!isfinite(gammacorr)) gammacorr = 0.;
    }
    gammacorr *= ARTIS_FOURPI * get_phixsprobability(K, e, i, l, t);
    if ((threadIdx.x & 63) == 0) K.C.corrphot[(int64_t)k * ntg + slot] = gammacorr;
  }
}

#endif
