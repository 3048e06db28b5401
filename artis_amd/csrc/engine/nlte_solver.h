// nlte_solver.h -- update_grid for the nebular options on the GPU (artis_gpu_update_grid_nlte, include/artis_gpu.h;
// SURVEY.md §8(f) row 4), the device side of oracle/nebular_update_grid.cc.
//
// The cell loop of the reference (one OpenMP thread per model cell, update_grid.cc:1012-1205) becomes a sequence of
// kernels over the listed cells, each kernel one step of solve_Te_nltepops for every cell still iterating:
//
//   k_nl_prepare     estimator normalisation, the LTE branch's T_J, the full-spectrum fit (radfield.cc:1136-1175)
//   k_nl_bfnorm      normalise_bf_estimators (radfield.cc:1306-1327), workitem = (cell, continuum)
//   k_nl_binfit      the per-bin fit (radfield.cc:1177-1291): one workitem per (cell, bin) running GSL Brent on the
//                    mean frequency, the Planck integrals by the GK61 rule on kT-sized panels (D14)
//   k_nl_bfheat      calculate_bfheatingcoeffs with NO_LUT_BFHEATING (thermalbalance.cc:60-187): one wave per (cell,
//                    ionising level), its targets' qag integrals in order
//   Spencer-Fano     (nonthermal.cc:2522-2713) one cell at a time, the SFPTS x SFPTS system in HBM (128 MiB):
//     k_sf_decide      the skip / keep / solve decision and the skip path's defaults
//     k_sf_ions        ion populations of the cell, the ions the matrix includes
//     k_sf_matrix      every matrix element in one workitem, the reference's additions in its order (loss term, then
//                      per included ion its excitation band and its shells' ionisation and Auger terms), written
//                      column-major (MT[j * n + i] = M[i][j]) for the column-oriented solves
//     k_sf_backsub     the upper-triangular solve, one workgroup, blocked by 64 columns; every x_i still receives its
//                      subtractions one at a time in descending column order (the column-oriented order, D11)
//     k_sf_residual_*  A x - b: serial sums over 256-column chunks per (row, chunk), then the chunks in order
//     k_sf_best        gsl_linalg_LU_refine's bookkeeping: x -= work, idamax, the best solution so far
//     k_sf_dots        analyse_sf_solution's dot products (one workitem per shell / excitation transition, serial sums)
//     k_sf_combine     the per-ion sums of analyse_sf_solution and calculate_eff_ionpot_auger_rates
//   k_nl_ntrates     nt_ionization_ratecoeff of every ion, the thermal balance's deposition heating
//   k_te_solve       call_T_e_finder in mode 1 (te_solver.h)
//   k_levelpops, k_bfcells, k_corrphot_integral (engine.hip, qag.h) on the solver's state: the populations and
//                    corrected photoionisation coefficients of the NLTE rate matrix
//   k_nl_slpf        superlevel partition functions (nltepop.cc:832-850)
//   k_nl_matrix      the rate matrix of every (cell, element), a workitem per column: the five process matrices of
//                    nltepop.cc:421-591 column by column in the reference's accumulation order, summed, normalised
//   k_nl_lu          LU with partial pivoting + iterative refinement (nltepop.cc:656-796), a workgroup per (cell,
//                    element)
//   k_nl_store       nltepop.cc:1040-1113, precalculate_partfuncts, calculate_electron_densities, the convergence test
#pragma once

#define NL_MAX_AUGER ARTIS_NT_MAX_AUGER
#define NL_A1 (NL_MAX_AUGER + 1)
#define SF_WG 1024   // k_sf_backsub workgroup
#define SF_NMAX 8192 // SFPTS bound of k_sf_backsub's LDS vector

// the listed cells' state (device copies of artis_nlte_cells, by mgi) and per-call scratch
struct NlDev {
  int32_t np, ncells;
  const int32_t *mgi;  // [ncells]
  int32_t nts, num_lte_timesteps, initial_iteration, nprocs, do_rlc_est, nt_on, sf_on;
  double deltat, tratmid, T_min, T_max, T_R_min, T_R_max;
  const float *rho, *abund, *meanw;
  const double *vol;
  const int16_t *thick;
  const double *dep;
  const double *J, *nuJ, *ffraw, *bfraw, *binJ, *binnuJ;
  const int64_t *bincount;
  float *TR, *W, *TJ, *Te, *nne, *nnetot, *gp, *pf;
  double *nlte;
  float *binTR, *binW, *bfrate;
  float *nt_fh, *nt_fi, *nt_fe, *nt_nneper;
  int32_t *nt_tls;
  float *nt_effion;
  double *nt_fracdep;
  float *nt_prob, *nt_ionen;
  double *ntY;
  double *ffheat, *hdep, *prevTe;  // [np] scratch: normalised ff heating, deposition heating, T_e before the finder
  int32_t *fail;                   // [2]: first failing cell (mgi + 1), reason
};

enum : int32_t { NLF_BINFIT = 1, NLF_BFHEAT = 2, NLF_BINDING = 3, NLF_POPS = 4, NLF_TE = 5 };
DEVFN void nl_fail(const NlDev &N, int mgi, int why) {
  if (atomicCAS(N.fail, 0, mgi + 1) == 0) N.fail[1] = why;
}

// grid.cc:231-236 / atomic.cc:58-66
DEVFN double nl_elem_numberdens(const Ctx &K, const NlDev &N, int mgi, int e) {
  const int64_t k = (int64_t)mgi * K.T.nelements + e;
  return N.abund[k] / N.meanw[k] * (double)N.rho[mgi];
}
DEVFN double nl_get_nntot(const Ctx &K, const NlDev &N, int mgi) {
  double nntot = 0.;
  for (int e = 0; e < K.T.nelements; e++) nntot += nl_elem_numberdens(K, N, mgi, e);
  return nntot;
}
// ltepop.cc:307-327, 558-564
DEVFN double nl_gpop(const Ctx &K, const NlDev &N, int mgi, int e, int ui) {
  const double nn = N.gp[(int64_t)mgi * K.T.nions_total + ui];
  if (nn < K.R.minpop) return N.abund[(int64_t)mgi * K.T.nelements + e] > 0 ? K.R.minpop : 0.;
  return nn;
}
DEVFN double nl_ionstagepop(const Ctx &K, const NlDev &N, int mgi, int e, int ui) {
  return nl_gpop(K, N, mgi, e, ui) * N.pf[(int64_t)mgi * K.T.nions_total + ui] /
         (double)K.T.level_stat_weight[K.T.ion_uniqueleveloffset[ui]];
}
DEVFN double nl_estimator_normfactor(const NlDev &N, int mgi) {
  const double deltaV = N.vol[mgi] * pow(N.tratmid, 3);
  return 1 / deltaV / N.deltat / N.nprocs;
}

// ---------------------------------------------------------------------------------------- preparation
// update_grid.cc:1104-1150 for one listed cell: the LTE branch's radiation field, or the normalised estimators and
// radfield::set_params_fullspec
__global__ void k_nl_prepare(NlDev N) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= N.ncells) return;
  const int mgi = N.mgi[k];
  const double estimator_normfactor = nl_estimator_normfactor(N, mgi);
  const double estimator_normfactor_over4pi = ARTIS_ONEOVER4PI * estimator_normfactor;
  const double J = N.J[mgi] * estimator_normfactor_over4pi;
  if (N.initial_iteration || N.thick[mgi] == 1) {
    double T_J = pow(J * ARTIS_PI / ARTIS_STEBO, 1. / 4.);
    if (!isfinite(T_J))
      T_J = N.TR[mgi];
    else if (T_J > N.T_max)
      T_J = N.T_max;
    else if (T_J < N.T_min)
      T_J = N.T_min;
    N.TR[mgi] = T_J;
    N.Te[mgi] = T_J;
    N.TJ[mgi] = T_J;
    N.W[mgi] = 1;
    return;
  }
  const double nuJ = N.nuJ[mgi] * estimator_normfactor_over4pi;
  N.ffheat[mgi] = N.ffraw[mgi] * estimator_normfactor;
  const double nubar = nuJ / J;
  if (isfinite(nubar) && nubar != 0.) {
    float T_J = pow(J * ARTIS_PI / ARTIS_STEBO, 1 / 4.);
    if (T_J > N.T_max)
      T_J = N.T_max;
    else if (T_J < N.T_min)
      T_J = N.T_min;
    N.TJ[mgi] = T_J;
    float T_R = ARTIS_H * nubar / ARTIS_KB / 3.832229494;
    if (T_R > N.T_max)
      T_R = N.T_max;
    else if (T_R < N.T_min)
      T_R = N.T_min;
    N.TR[mgi] = T_R;
    N.W[mgi] = J * ARTIS_PI / ARTIS_STEBO / pow((double)T_R, 4);
  }
}
// radfield.cc:1306-1327 normalise_bf_estimators for the listed non-LTE cells (list = mgi)
__global__ void k_nl_bfnorm(Ctx K, NlDev N, const int32_t *list, int nlist) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nb = K.T.nbf;
  if (idx >= (int64_t)nlist * nb) return;
  const int mgi = list[idx / nb];
  const int64_t q = (int64_t)mgi * nb + idx % nb;
  N.bfrate[q] = N.bfraw[q] * (nl_estimator_normfactor(N, mgi) / ARTIS_H);
}

// radfield.cc:945-979 planck_integral: the reference integrates the Planck function over a bin with GSL qag
// (GK61, epsrel 1e-10).  The integrand is analytic on the whole bin, so the engine evaluates the integral directly
// with the same 61-point Kronrod rule on panels at most 24 kT/h wide (deviation D14; the rule integrates e^-x x^3
// over such a panel to ~1e-30): on a bin qag accepts after its
// first rule this is that rule's value, otherwise it agrees with qag's result to qag's 1e-10 tolerance.  Per lane, no
// workspace; contributions beyond 800 kT/h above the lower edge (e^-800 of the integrand there) are dropped.
DEVFN double nl_planck_integral(double T_R, double nu_lower, double nu_upper, bool times_nu) {
  auto f = [&](double nu) {
    double integrand = ARTIS_TWOHOVERCLIGHTSQUARED * pow(nu, 3) / (expm1(ARTIS_HOVERKB * nu / T_R));
    if (times_nu) integrand *= nu;
    return integrand;
  };
  const double dnu_kT = T_R / ARTIS_HOVERKB;  // nu of one kT / h
  double b_end = nu_upper;
  if (b_end > nu_lower + 800. * dnu_kT) b_end = nu_lower + 800. * dnu_kT;
  const int npan = (int)fmin(fmax(ceil((b_end - nu_lower) / (24. * dnu_kT)), 1.), 40.);
  const double width = (b_end - nu_lower) / npan;
  double integral = 0.;
  for (int p = 0; p < npan; p++) {
    const double a = nu_lower + p * width;
    const double b = (p == npan - 1) ? b_end : a + width;
    const double center = 0.5 * (a + b), half_length = 0.5 * (b - a);
    double result_kronrod = f(center) * c_qk61_wgk[30];
    for (int j = 0; j < 30; j++) {
      const double abscissa = half_length * c_qk61_xgk[j];
      result_kronrod += c_qk61_wgk[j] * (f(center - abscissa) + f(center + abscissa));
    }
    const double panel = result_kronrod * half_length;
    integral += panel;
    if (p > 0 && panel <= 1e-18 * integral) break;  // past the Wien peak: the rest is below the last bit
  }
  return integral;
}
DEVFN double nl_bin_nu_lower(const Ctx &K, int b) { return b > 0 ? K.T.rf_nu_upper[b - 1] : K.T.rf_nu_lower_first; }

// radfield.cc:1177-1291 fit_parameters' bin loop, one workitem per (listed non-LTE cell, bin): GSL Brent on the mean
// frequency of a dilute Planck function (radfield.cc:1070-1133 find_T_R), the bin's dilution factor
__global__ __launch_bounds__(64) void k_nl_binfit(const Ctx *__restrict__ Kp, const NlDev *__restrict__ Np,
                                                  const int32_t *list, int nlist) {
  const Ctx &K = *Kp;
  const NlDev &N = *Np;
  const int nb = K.T.rf_nbins;
  const int64_t item = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (item >= (int64_t)nlist * nb) return;
  const int mgi = list[item / nb];
  const int b = (int)(item % nb);
  const int64_t mb = (int64_t)mgi * nb + b;
  const double J_normfactor = ARTIS_ONEOVER4PI * nl_estimator_normfactor(N, mgi);
  const double nu_lower = nl_bin_nu_lower(K, b), nu_upper = K.T.rf_nu_upper[b];
  const double J_bin = N.binJ[mb] * J_normfactor;
  float T_R_bin = -1.0;
  double W_bin = -1.0;
  if (N.bincount[mb] > 0) {
    const double nu_bar = (N.binnuJ[mb] * J_normfactor) / J_bin;
    auto delta_nu_bar = [&](double T_R) {
      const double nu_times_planck = nl_planck_integral(T_R, nu_lower, nu_upper, true);
      const double planck = nl_planck_integral(T_R, nu_lower, nu_upper, false);
      return nu_times_planck / planck - nu_bar;
    };
    const double T_R_min = N.T_R_min, T_R_max = N.T_R_max;
    double delta_nu_bar_min = delta_nu_bar(T_R_min);
    double delta_nu_bar_max = delta_nu_bar(T_R_max);
    if (!isfinite(delta_nu_bar_min) || !isfinite(delta_nu_bar_max)) delta_nu_bar_max = delta_nu_bar_min = -1;
    double T_R = 0.;
    bool bad = false;
    if (delta_nu_bar_min * delta_nu_bar_max < 0) {
      TeBrent s;
      if (te_brent_set(s, delta_nu_bar, T_R_min, T_R_max) != 0) bad = true;
      int iteration_num = 0, status = 1;
      while (!bad && status == 1 && iteration_num < 100) {
        iteration_num++;
        if (te_brent_iterate(s, delta_nu_bar) != 0) {
          bad = true;
          break;
        }
        T_R = s.root;
        status = te_test_interval(s.x_lower, s.x_upper, 0., 1e-4);
      }
    } else if (delta_nu_bar_max < 0) {
      T_R = T_R_max;
    } else {
      T_R = T_R_min;
    }
    if (bad) {
      nl_fail(N, mgi, NLF_BINFIT);
      T_R = 0.;
    }
    T_R_bin = T_R;
    if (b == nb - 1) T_R_bin = N.Te[mgi];
    double planck_integral_result = nl_planck_integral(T_R_bin, nu_lower, nu_upper, false);
    W_bin = J_bin / planck_integral_result;
    if (W_bin > 1e4) {
      planck_integral_result = nl_planck_integral(N.T_R_max, nu_lower, nu_upper, false);
      W_bin = J_bin / planck_integral_result;
      if (W_bin > 1e4) {
        T_R_bin = -99.0;
        W_bin = 0.;
      } else {
        T_R_bin = N.T_R_max;
      }
    }
  } else {
    T_R_bin = 0.;
    W_bin = 0.;
  }
  N.binTR[mb] = T_R_bin;
  N.binW[mb] = W_bin;
}

// thermalbalance.cc:60-132 calculate_bfheatingcoeff of one target (not inlined, see nl_planck_integral)
DEVNI double nl_bfheat_target(const Ctx &K, int mgi, int e, int i, int l, int t, float T_R, double *al, double *bl,
                              double *rl, QagLists Q, int32_t *lev, double *s_f) {
  const float *xs = level_photoion_xs(K, e, i, l);
  const double E_threshold = get_phixs_threshold(K, e, i, l, t);
  const double nu_threshold = ARTIS_ONEOVERH * E_threshold;
  const double nu_max_phixs = nu_threshold * K.T.last_phixs_nuovernuedge;
  auto integrand = [&](double nu) {
    const float sigma_bf = (float)photoionization_crosssection_fromtable(K, xs, nu_threshold, nu);
    return sigma_bf * (1 - nu_threshold / nu) * radfield_J(K, mgi, nu) * (1 - exp(-ARTIS_HOVERKB * nu / T_R));
  };
  double bfheating = 0., error = 0.;
  qag61(integrand, nu_threshold, nu_max_phixs, 0., 1e-3, al, bl, rl, Q, lev, s_f, &bfheating, &error);
  bfheating *= ARTIS_FOURPI * get_phixsprobability(K, e, i, l, t);
  return bfheating;
}
// thermalbalance.cc:60-132, 141-187 (NO_LUT_BFHEATING): the bf-heating coefficient of every ionising level of the
// heating sum (hb_ul) for the listed non-LTE cells; one wave per (cell, level), grid-strided.  Context K: the
// solver's state (its fitted bins, T_R).
__global__ __launch_bounds__(64) void k_nl_bfheat(const Ctx *__restrict__ Kp, const NlDev *__restrict__ Np,
                                                  const int32_t *list, int nlist, const int32_t *hb_ul, int nhb,
                                                  double *hbc, QagWs ws) {
  const Ctx &K = *Kp;
  const NlDev &N = *Np;
  __shared__ double s_f[64];
  __shared__ double s_el[QAG_LDS];
  __shared__ int32_t s_ord[QAG_LDS];
  const int64_t total = (int64_t)nlist * nhb;
  const int64_t wbase = (int64_t)blockIdx.x * QAG_LIMIT;
  double *al = ws.alist + wbase, *bl = ws.blist + wbase, *rl = ws.rlist + wbase;
  int32_t *lev = ws.level + wbase;
  const QagLists Q{s_el, s_ord, ws.elist + wbase, ws.order + wbase};
  double *sf = s_f;
  for (int64_t item = blockIdx.x; item < total; item += gridDim.x) {
    const int kk = (int)(item % nlist);
    const int j = (int)(item / nlist);
    const int mgi = list[kk];
    const int ul = hb_ul[j];
    const int ui = K.T.level_ui[ul];
    const int e = K.T.ion_element[ui];
    const int i = ui - K.T.elem_uniqueionoffset[e];
    const int l = ul - K.T.ion_uniqueleveloffset[ui];
    double bfheatingcoeff = 0.;
    if (N.abund[(int64_t)mgi * K.T.nelements + e] > 0.01) {  // minelfrac
      const float T_R = N.TR[mgi];
      for (int t = 0; t < get_nphixstargets(K, e, i, l); t++)
        bfheatingcoeff += nl_bfheat_target(K, mgi, e, i, l, t, T_R, al, bl, rl, Q, lev, sf);
      if (!isfinite(bfheatingcoeff) && (threadIdx.x & 63) == 0) nl_fail(N, mgi, NLF_BFHEAT);
    }
    if ((threadIdx.x & 63) == 0) hbc[(int64_t)j * nlist + kk] = bfheatingcoeff;
  }
}

// ------------------------------------------------------------------------------------------- Spencer-Fano
// host-built tables (engine.hip): the energy grid with its host-libm transcendentals, the shells of every ion
// (collion.txt entries matching (Z, ionstage), nonthermal.cc:183-437) with their cross sections and the atan
// terms of sfmatrix_add_ionization, the excitation transitions (lower < NTEXCITATION_MAXNLEVELS_LOWER, upper <
// NTEXCITATION_MAXNLEVELS_UPPER, with a cross section)
struct SfDev {
  int32_t n, band;
  double emin, emax, DE, E_init_ev;
  const double *envec, *logenvec, *pw2, *rhs;  // pw2[j] = pow(envec[j] * EV, -2); rhs: source integral to SF_EMAX
  const int32_t *ion_sh_off;                   // [ni + 1] CSR of shell records
  const int32_t *sh_k, *sh_xsstart, *sh_augerstop;
  const double *sh_ionpot_ev, *sh_J;  // ionisation potential [eV], get_J (nonthermal.cc:994-1007)
  const double *sh_xs, *sh_ieu, *sh_atn, *sh_ie2;  // [nsh * n]
  const double *sh_prob;                           // [nsh * NL_A1] prob_num_auger
  const int32_t *ion_tr_off;                       // [ni + 1] CSR of excitation transitions
  const int32_t *tr_ul, *tr_kind, *tr_start, *tr_build;
  const double *tr_cf, *tr_logeps, *tr_eps_ev, *tr_eps;
  const double *ion_binding;      // [ni] get_mean_binding_energy
  const int32_t *ion_binding_ok;  // [ni] 0: the reference aborts if the work-function approximation is needed
  int32_t nsh, nitems;            // shell records; shells + transitions (k_sf_dots)
  const int32_t *anumber;         // [nelements]
  // a batch of cells solved together, slot q: the cell's active position bat_a[q] and model cell bat_mgi[q]
  const int32_t *bat_a, *bat_mgi;
  double *nnion;    // [q * ni]
  int32_t *incl;    // [q * ni]
  double *tot_nion; // [q]
  double *MT;       // [q * n * n] column-major
  double *x, *best, *work, *res;  // [q * n]
  double *errbest;  // [q]
  double *dots;     // [q * nitems]
  double *part;     // [q * nchunks * n] k_sf_residual_part
  int32_t *solve;   // [ncells] k_sf_decide's verdict
};

// nonthermal.cc:757-789
DEVFN int sf_lteq(const SfDev &S, double energy_ev) {
  const int index = (int)floor((energy_ev - S.emin) / S.DE);
  return index < 0 ? 0 : (index > S.n - 1 ? S.n - 1 : index);
}
// nonthermal.cc:820-840 electron_loss_rate [erg / cm]
DEVFN double sf_electron_loss_rate(double energy, double nne) {
  if (energy <= 0.) return 0;
  const double boostfactor = 1.;
  const double omegap = sqrt(4 * ARTIS_PI * nne * pow(ARTIS_QE, 2) / ARTIS_ME);
  const double zetae = ARTIS_H * omegap / 2 / ARTIS_PI;
  if (energy > 14 * ARTIS_EV) return boostfactor * nne * 2 * ARTIS_PI * pow(ARTIS_QE, 4) / energy * log(2 * energy / zetae);
  const double v = sqrt(2 * energy / ARTIS_ME);
  const double eulergamma = 0.577215664901532;
  return boostfactor * nne * 2 * ARTIS_PI * pow(ARTIS_QE, 4) / energy *
         log(ARTIS_ME * pow(v, 3) / (eulergamma * pow(ARTIS_QE, 2) * omegap));
}
// nonthermal.cc:872-929 get_xs_excitation_vector at one energy (0 below the start index)
DEVFN double sf_xs_exc(const SfDev &S, int t, int j) {
  if (j < S.tr_start[t]) return 0.;
  if (S.tr_kind[t] == 0) return S.tr_cf[t] * S.pw2[j];
  const double logU = S.logenvec[j] - S.tr_logeps[t];
  const double g_bar = 0.28 * logU + 0.15;
  return S.tr_cf[t] * g_bar / S.envec[j];
}

// nonthermal.cc:2522-2560 the skip / keep decision; solve[k] = 1: solve now (nneperion / timestep stored)
__global__ void k_sf_decide(Ctx K, NlDev N, SfDev S, const int32_t *act, int nact) {
  const int a = blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= nact) return;
  const int mgi = act[a];
  const int ni = K.T.nions_total;
  S.solve[a] = 0;
  bool skip_solution = false;
  if (N.nts < N.num_lte_timesteps + 1)
    skip_solution = true;
  else if (N.dep[mgi] / ARTIS_EV < 0.)
    skip_solution = true;
  if (skip_solution) {
    N.nt_fh[mgi] = 0.97;
    N.nt_fi[mgi] = 0.03;
    N.nt_fe[mgi] = 0.;
    N.nt_nneper[mgi] = -1.;
    N.nt_tls[mgi] = -1;
    for (int u = 0; u < ni; u++) {  // zero_all_effionpot (nonthermal.cc:439-460)
      N.nt_effion[(int64_t)mgi * ni + u] = 0.;
      float *pr = N.nt_prob + ((int64_t)mgi * ni + u) * NL_A1;
      float *ie = N.nt_ionen + ((int64_t)mgi * ni + u) * NL_A1;
      pr[0] = 1.;
      ie[0] = 1.;
      for (int q = 1; q < NL_A1; q++) {
        pr[q] = 0.;
        ie[q] = 0.;
      }
    }
    return;
  }
  const float nne = N.nne[mgi];
  const double nne_per_ion = nne / nl_get_nntot(K, N, mgi);
  const double nne_per_ion_last = N.nt_nneper[mgi];
  const double nne_per_ion_fracdiff = fabs((nne_per_ion_last / nne_per_ion) - 1.);
  const int timestep_last_solved = N.nt_tls[mgi];
  if ((nne_per_ion_fracdiff < 0.05) && (N.nts - timestep_last_solved <= 0) && timestep_last_solved > N.num_lte_timesteps)
    return;
  N.nt_nneper[mgi] = nne_per_ion;
  N.nt_tls[mgi] = N.nts;
  S.solve[a] = 1;
}

// the ion populations of the cell being solved and the ions solve_spencerfano includes (nonthermal.cc:2630-2640)
__global__ void k_sf_ions(Ctx K, NlDev N, SfDev S, int nbat) {
  const int ni = K.T.nions_total;
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= nbat * ni) return;
  const int q = idx / ni, ui = idx % ni;
  const int mgi = S.bat_mgi[q];
  const int e = K.T.ion_element[ui];
  const double tot_nion = nl_get_nntot(K, N, mgi);
  const double nnion = nl_ionstagepop(K, N, mgi, e, ui);
  S.nnion[idx] = nnion;
  S.incl[idx] = !(nnion < 1.e-8 * tot_nion);  // MINFRAC
  if (ui == 0) S.tot_nion[q] = tot_nion;
}

// nonthermal.cc:2617-2674 with sfmatrix_add_excitation (2282-2341) and sfmatrix_add_ionization (2343-2459): matrix
// element (i, j >= i) in one workitem, its additions in the reference's order.  Grid: x over rows i, y = column j,
// z = batch slot.  pops0: the active cells' level populations (k_levelpops of the solver state).
__global__ __launch_bounds__(256) void k_sf_matrix(Ctx K, NlDev N, SfDev S, const double *__restrict__ pops0) {
  const int j = blockIdx.y;
  const int q = blockIdx.z;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int n = S.n;
  if (i >= n) return;
  if (i > j) return;  // the strictly lower part is never read
  const int mgi = S.bat_mgi[q];
  const double *pops = pops0 + (int64_t)S.bat_a[q] * K.T.nlevels_total;
  const double *nnion_q = S.nnion + (int64_t)q * K.T.nions_total;
  const int32_t *incl_q = S.incl + (int64_t)q * K.T.nions_total;
  double *out = S.MT + (int64_t)q * n * n + (int64_t)j * n + i;
  const double DE = S.DE;
  const double en = S.envec[i];
  double m = 0.;
  if (i == j) m += sf_electron_loss_rate(en * ARTIS_EV, (float)N.nne[mgi]) / ARTIS_EV;
  const double endash = S.envec[j];
  const bool in_band = j - i <= S.band;
  for (int ui = 0; ui < K.T.nions_total; ui++) {
    if (!incl_q[ui]) continue;
    const double nnion = nnion_q[ui];
    // excitation: the band j - i <= max stop - start of the ion's transitions
    if (in_band) {
      for (int t = S.ion_tr_off[ui]; t < S.ion_tr_off[ui + 1]; t++) {
        if (!S.tr_build[t]) continue;
        const double eps_ev = S.tr_eps_ev[t];
        const int stopindex = sf_lteq(S, en + eps_ev);
        const int startindex = i > S.tr_start[t] ? i : S.tr_start[t];
        if (j >= startindex && j < stopindex) {
          m += pops[S.tr_ul[t]] * (sf_xs_exc(S, t, j) * DE);
        } else if (j == stopindex) {
          const double delta_en_actual = (en + eps_ev - S.envec[stopindex]);
          m += pops[S.tr_ul[t]] * (sf_xs_exc(S, t, stopindex) * DE) * delta_en_actual / DE;
        }
      }
    }
    // ionisation (ions below the top one), shells in collion order; then the shell's Auger term
    const int e = K.T.ion_element[ui];
    if (ui - K.T.elem_uniqueionoffset[e] >= K.T.elem_nions[e] - 1) continue;
    for (int r = S.ion_sh_off[ui]; r < S.ion_sh_off[ui + 1]; r++) {
      const int xsstart = S.sh_xsstart[r];
      const double ionpot_ev = S.sh_ionpot_ev[r];
      const double Jsh = S.sh_J[r];
      const double *xs = S.sh_xs + (int64_t)r * n;
      const double *ieu = S.sh_ieu + (int64_t)r * n;
      const double prefactor = j >= xsstart ? xs[j] * nnion / S.sh_atn[(int64_t)r * n + j] : 0.;
      // the first integral (nonthermal.cc:2390-2402)
      if (j >= (i > xsstart ? i : xsstart)) {
        const double epsilon_lower = fmax(endash - en, ionpot_ev);
        const double int_eps_lower = atan((epsilon_lower - ionpot_ev) / Jsh);
        if (int_eps_lower <= ieu[j]) m += prefactor * (ieu[j] - int_eps_lower) * DE;
      }
      // the second integral (nonthermal.cc:2405-2419; D10: not below xsstartindex)
      if (2 * en + ionpot_ev <= S.emax) {
        const int secondintegralstartindex = sf_lteq(S, 2 * en + ionpot_ev);
        if (j >= (secondintegralstartindex > xsstart ? secondintegralstartindex : xsstart)) {
          const double int_eps_lower2 = S.sh_ie2[(int64_t)r * n + i];
          if (int_eps_lower2 <= ieu[j]) m -= prefactor * (ieu[j] - int_eps_lower2) * DE;
        }
      }
      // SF_AUGER_CONTRIBUTION_ON (nonthermal.cc:2421-2457, SF_AUGER_CONTRIBUTION_DISTRIBUTE_EN false)
      if (i < S.sh_augerstop[r] && j >= (i > xsstart ? i : xsstart)) m -= nnion * xs[j];
    }
  }
  *out = m;
}

// Upper-triangular solve M v = v in place (GSL LU_svx with the identity permutation: the unit-lower solve is the
// identity; D11's column-oriented back substitution).  One workgroup; v staged in LDS.  Columns in blocks of 64 from
// the right: the block's 64 x 64 diagonal tile is staged in LDS by the whole workgroup, wave 0 finishes the block's own
// unknowns from it (lane r holds x_{j0+r}; for each column j, top-down, x_j is divided by the diagonal and broadcast,
// the block rows above it updated), then every row above the block receives the block's 64 subtractions in
// descending column order -- per x_i the same sequence as the unblocked loop.
__global__ __launch_bounds__(SF_WG) void k_sf_backsub(const double *__restrict__ MT0, int n, double *v0) {
  const double *MT = MT0 + (int64_t)blockIdx.x * n * n;  // one workgroup per batch slot
  double *v = v0 + (int64_t)blockIdx.x * n;
  __shared__ double x[SF_NMAX];
  __shared__ double tile[64 * 65];  // tile[c * 65 + r] = M[j0 + r][j0 + c], padded against bank conflicts
  for (int i = threadIdx.x; i < n; i += SF_WG) x[i] = v[i];
  const int nblk = (n + 63) / 64;
  for (int jb = nblk - 1; jb >= 0; jb--) {
    const int j0 = jb * 64;
    const int j1 = min(j0 + 64, n);
    for (int q = threadIdx.x; q < 64 * 64; q += SF_WG) {
      const int c = q >> 6, r = q & 63;
      if (j0 + c < j1 && r <= c) tile[c * 65 + r] = MT[(int64_t)(j0 + c) * n + j0 + r];
    }
    __syncthreads();
    if (threadIdx.x < 64) {
      const int lane = threadIdx.x;
      const int r = j0 + lane;
      double xr = r < j1 ? x[r] : 0.;
      for (int j = j1 - 1; j >= j0; j--) {
        const int c = j - j0;
        if (lane == c) xr = xr / tile[c * 65 + c];
        const double xj = __shfl(xr, c, 64);
        if (lane < c) xr -= tile[c * 65 + lane] * xj;
      }
      if (r < j1) x[r] = xr;
    }
    __syncthreads();
    // rows above the block: up to 4 rows per workitem as independent chains, the column loads unrolled
    for (int i0 = threadIdx.x; i0 < j0; i0 += 4 * SF_WG) {
      double xr[4];
#pragma unroll
      for (int k = 0; k < 4; k++) xr[k] = (i0 + k * SF_WG < j0) ? x[i0 + k * SF_WG] : 0.;
#pragma unroll 8
      for (int j = j1 - 1; j >= j0; j--) {
        const double xj = x[j];
        const double *col = MT + (int64_t)j * n;
#pragma unroll
        for (int k = 0; k < 4; k++)
          if (i0 + k * SF_WG < j0) xr[k] -= col[i0 + k * SF_WG] * xj;
      }
#pragma unroll
      for (int k = 0; k < 4; k++)
        if (i0 + k * SF_WG < j0) x[i0 + k * SF_WG] = xr[k];
    }
    __syncthreads();
  }
  for (int i = threadIdx.x; i < n; i += SF_WG) v[i] = x[i];
}
// res = M x - b (gsl_blas_dgemv, beta -1): res_i = -b_i + sum_{j >= i} x_j M_ij.  The row sums are split into
// SF_RCHUNK-column chunks, each summed serially (k_sf_residual_part, workitem = (row, chunk): coalesced over the
// column-major matrix and enough waves to fill the chip), then the chunks added in column order (k_sf_residual_sum).
#define SF_RCHUNK 256
__global__ __launch_bounds__(256) void k_sf_residual_part(const double *__restrict__ MT0, int n,
                                                          const double *__restrict__ xv0, double *part0) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int c = blockIdx.y;
  if (i >= n) return;
  const int q = blockIdx.z;
  const int nch = (n + SF_RCHUNK - 1) / SF_RCHUNK;
  const double *MT = MT0 + (int64_t)q * n * n;
  const double *xv = xv0 + (int64_t)q * n;
  double *part = part0 + (int64_t)q * nch * n;
  const int ja = max(i, c * SF_RCHUNK), jb = min(n, (c + 1) * SF_RCHUNK);
  double temp = 0.;
#pragma unroll 8
  for (int j = ja; j < jb; j++) temp += xv[j] * MT[(int64_t)j * n + i];
  part[(int64_t)c * n + i] = temp;
}
__global__ __launch_bounds__(256) void k_sf_residual_sum(int n, const double *__restrict__ part0,
                                                         const double *__restrict__ b, double *res0) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int nch = (n + SF_RCHUNK - 1) / SF_RCHUNK;
  const int q = blockIdx.y;
  const double *part = part0 + (int64_t)q * nch * n;
  double *res = res0 + (int64_t)q * n;
  double temp = 0.;
  for (int c = i / SF_RCHUNK; c < nch; c++) temp += part[(int64_t)c * n + i];
  res[i] = -b[i] + temp;
}
// x += -1 * work (gsl_blas_daxpy in gsl_linalg_LU_refine)
__global__ void k_sf_axpy(int n, double *xv, const double *__restrict__ work) {
  const int64_t i = (int64_t)blockIdx.y * n + blockIdx.x * blockDim.x + threadIdx.x;
  if (blockIdx.x * blockDim.x + threadIdx.x < n) xv[i] += -1.0 * work[i];
}
// nonthermal.cc:2490-2510: error = |res| at gsl_blas_idamax (first index of the largest), the best x so far kept;
// errbest < 0: none yet.  One workgroup.
__global__ __launch_bounds__(1024) void k_sf_best(int n, const double *__restrict__ res0,
                                                  const double *__restrict__ xv0, double *best0, double *errbest0) {
  const int64_t off = (int64_t)blockIdx.x * n;  // one workgroup per batch slot
  const double *res = res0 + off, *xv = xv0 + off;
  double *best = best0 + off, *errbest = errbest0 + blockIdx.x;
  __shared__ double s_v[1024];
  __shared__ int s_i[1024];
  __shared__ int s_take;
  double amax = -1.;
  int imax = 0;
  for (int i = threadIdx.x; i < n; i += 1024) {
    const double a = fabs(res[i]);
    if (a > amax) {
      amax = a;
      imax = i;
    }
  }
  s_v[threadIdx.x] = amax;
  s_i[threadIdx.x] = imax;
  __syncthreads();
  for (int w = 512; w > 0; w >>= 1) {
    if (threadIdx.x < w) {
      const double a = s_v[threadIdx.x + w];
      const int ia = s_i[threadIdx.x + w];
      if (a > s_v[threadIdx.x] || (a == s_v[threadIdx.x] && ia < s_i[threadIdx.x])) {
        s_v[threadIdx.x] = a;
        s_i[threadIdx.x] = ia;
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const double error = fabs(res[s_i[0]]);
    s_take = (error < errbest[0] || errbest[0] < 0.);
    if (s_take) errbest[0] = error;
  }
  __syncthreads();
  if (s_take)
    for (int i = threadIdx.x; i < n; i += 1024) best[i] = xv[i];
}

// analyse_sf_solution's dot products (nonthermal.cc:1333-1360 calculate_nt_frac_ionization_shell: y . xs_shell;
// 1714-1744 calculate_nt_excitation_ratecoeff_perdeposition: xs_trans . y), one workitem each, serial in j
__global__ void k_sf_dots(SfDev S, const double *__restrict__ y0) {
  const int item = blockIdx.x * blockDim.x + threadIdx.x;
  if (item >= S.nitems) return;
  const int q = blockIdx.y;
  const double *y = y0 + (int64_t)q * S.n;
  const int nsh = S.nsh;
  double dot = 0.;
  if (item < nsh) {
    const double *xs = S.sh_xs + (int64_t)item * S.n;
    for (int j = 0; j < S.n; j++) dot += y[j] * xs[j];
  } else {
    const int t = item - nsh;
    for (int j = 0; j < S.n; j++) dot += sf_xs_exc(S, t, j) * y[j];
  }
  S.dots[(int64_t)q * S.nitems + item] = dot;
}

// nonthermal.cc:1311-1331 get_oneoverw (the ion's mean binding energy from the host, get_mean_binding_energy)
DEVFN double sf_oneoverw(const Ctx &K, const NlDev &N, const SfDev &S, int ui, int mgi, bool *bad) {
  double Zbar = 0.0;
  for (int ie = 0; ie < K.T.nelements; ie++) Zbar += N.abund[(int64_t)mgi * K.T.nelements + ie] * S.anumber[ie];
  const double Aconst = 1.33e-14 * ARTIS_EV * ARTIS_EV;
  if (!S.ion_binding_ok[ui]) *bad = true;
  const double binding = S.ion_binding[ui];
  return Aconst * binding / Zbar / (2 * 3.14159 * pow(ARTIS_QE, 4));
}

// nonthermal.cc:1996-2280 analyse_sf_solution (NT_EXCITATION_ON false, D12) with calculate_eff_ionpot_auger_rates
// (1430-1556) for one cell: the per-ion combination of k_sf_dots' products, one workitem, the reference's order
__global__ void k_sf_combine(Ctx K, NlDev N, SfDev S, const double *__restrict__ pops0, int nbat) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= nbat) return;
  const int mgi = S.bat_mgi[q];
  const double *pops = pops0 + (int64_t)S.bat_a[q] * K.T.nlevels_total;
  const int ni = K.T.nions_total;
  const double *dots = S.dots + (int64_t)q * S.nitems;
  const double DE = S.DE, E_init_ev = S.E_init_ev;
  const double tot_nion = S.tot_nion[q];
  double frac_excitation_total = 0., frac_ionization_total = 0.;
  bool bad = false;
  for (int e = 0; e < K.T.nelements; e++) {
    const int nions = K.T.elem_nions[e];
    for (int i = 0; i < nions; i++) {
      const int u = uion(K, e, i);
      const double nnion = S.nnion[(int64_t)q * ni + u];
      if (nnion <= 0.) continue;
      // calculate_eff_ionpot_auger_rates
      float *prob = N.nt_prob + ((int64_t)mgi * ni + u) * NL_A1;
      float *ionen = N.nt_ionen + ((int64_t)mgi * ni + u) * NL_A1;
      const double X_ion = nnion / tot_nion;
      double eta_nauger_ionize_over_ionpot_sum[NL_A1], eta_nauger_ionize_sum[NL_A1];
      for (int q = 0; q < NL_A1; q++) {
        eta_nauger_ionize_over_ionpot_sum[q] = 0.;
        prob[q] = 0.;
        eta_nauger_ionize_sum[q] = 0.;
        ionen[q] = 0.;
      }
      double eta_over_ionpot_sum = 0., eta_sum = 0.;
      const int r0 = S.ion_sh_off[u], r1 = S.ion_sh_off[u + 1];
      for (int r = r0; r < r1; r++) {
        const double frac_ionization_shell = nnion * S.sh_ionpot_ev[r] * (dots[r] * DE) / E_init_ev;
        eta_sum += frac_ionization_shell;
        const double ionpot_shell = S.sh_ionpot_ev[r] * ARTIS_EV;
        const double eta_over_ionpot = frac_ionization_shell / ionpot_shell;
        eta_over_ionpot_sum += eta_over_ionpot;
        for (int q = 0; q < NL_A1; q++) {
          eta_nauger_ionize_over_ionpot_sum[q] += eta_over_ionpot * S.sh_prob[r * NL_A1 + q];
          eta_nauger_ionize_sum[q] += frac_ionization_shell * S.sh_prob[r * NL_A1 + q];
        }
      }
      const int matching = r1 - r0;
      if (NL_MAX_AUGER > 0 && matching > 0) {
        if (i < nions - 1) {
          for (int q = 0; q < NL_A1; q++) {
            if (i + 1 + q < nions) {
              prob[q] = eta_nauger_ionize_over_ionpot_sum[q] / eta_over_ionpot_sum;
              ionen[q] = eta_nauger_ionize_sum[q] / eta_sum;
            } else {
              prob[nions - 1 - i - 1] += eta_nauger_ionize_over_ionpot_sum[q] / eta_over_ionpot_sum;
              ionen[nions - 1 - i - 1] += eta_nauger_ionize_sum[q] / eta_sum;
              prob[q] = 0;
              ionen[q] = 0.;
            }
          }
        }
      } else {
        prob[0] = 1.;
        ionen[0] = 1.;
      }
      if (matching > 0) {
        double eff_ionpot = X_ion / eta_over_ionpot_sum;
        if (!isfinite(eff_ionpot)) eff_ionpot = 0.;
        N.nt_effion[(int64_t)mgi * ni + u] = eff_ionpot;
      } else {
        N.nt_effion[(int64_t)mgi * ni + u] = 1. / sf_oneoverw(K, N, S, u, mgi, &bad);
      }
      // the ion's ionisation and excitation fractions
      double frac_ionization_ion = 0., frac_excitation_ion = 0.;
      for (int r = r0; r < r1; r++) frac_ionization_ion += nnion * S.sh_ionpot_ev[r] * (dots[r] * DE) / E_init_ev;
      if (i < nions - 1) {
        N.nt_fracdep[(int64_t)mgi * ni + u] = frac_ionization_ion;
        frac_ionization_total += frac_ionization_ion;
      } else {
        N.nt_fracdep[(int64_t)mgi * ni + u] = 0.;
      }
      for (int t = S.ion_tr_off[u]; t < S.ion_tr_off[u + 1]; t++) {
        const double nnlevel = pops[S.tr_ul[t]];
        const double ratecoeff = (dots[S.nsh + t] * DE) / E_init_ev / ARTIS_EV;
        const double nt_frac_excitation_perlevelpop = S.tr_eps[t] * ratecoeff;
        frac_excitation_ion += nnlevel * nt_frac_excitation_perlevelpop;
      }
      if (frac_excitation_ion > 1. || !isfinite(frac_excitation_ion)) frac_excitation_ion = 0.;
      frac_excitation_total += frac_excitation_ion;
    }
  }
  N.nt_fe[mgi] = frac_excitation_total;
  N.nt_fi[mgi] = frac_ionization_total;
  N.nt_fh[mgi] = 1. - frac_excitation_total - frac_ionization_total;
  if (bad) nl_fail(N, mgi, NLF_BINDING);
}

// nonthermal.cc:1684-1712 nt_ionization_ratecoeff of every ion (NT_SOLVE_SPENCERFANO) into the state the rate matrix
// reads; the deposition heating of the thermal balance (thermalbalance.cc:373-376); T_e before call_T_e_finder
__global__ void k_nl_ntrates(Ctx K, NlDev N, SfDev S, const int32_t *act, int nact) {
  const int a = blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= nact) return;
  const int mgi = act[a];
  N.prevTe[mgi] = N.Te[mgi];
  N.hdep[mgi] = (N.do_rlc_est == 3) ? N.dep[mgi] * (double)N.nt_fh[mgi] : 0.;
  if (!N.nt_on) return;
  const int ni = K.T.nions_total;
  const double deposition_rate_density = N.dep[mgi];
  bool bad = false;
  for (int e = 0; e < K.T.nelements; e++)
    for (int i = 0; i < K.T.elem_nions[e]; i++) {
      const int u = uion(K, e, i);
      double Y = 0.;
      if (i < K.T.elem_nions[e] - 1) {
        if (deposition_rate_density > 0.)
          Y = deposition_rate_density / nl_get_nntot(K, N, mgi) / N.nt_effion[(int64_t)mgi * ni + u];
        if (!isfinite(Y) || Y <= 0)
          Y = deposition_rate_density / nl_get_nntot(K, N, mgi) * sf_oneoverw(K, N, S, u, mgi, &bad);
      }
      N.ntY[(int64_t)mgi * ni + u] = Y;
    }
  if (bad) nl_fail(N, mgi, NLF_BINDING);
}

// ------------------------------------------------------------------------------------------ NLTE populations
// per (cell, element) rate-matrix layout: a cell's matrices / vectors back to back, one element after another
struct NlMat {
  int32_t cell1;              // sum over elements of D_e
  int64_t cell2;              // sum of D_e^2
  const int32_t *el_D, *el_off1;
  const int64_t *el_off2;
  const int32_t *col_e, *col_ion, *col_l0, *col_l1;  // [cell1] per column: element, ion, level range
  double t_mid;
  double *A, *LU, *P;         // [chunk * cell2], P: [chunk * 5 * cell2]
  double *b, *norm, *pv, *xv, *best, *work, *res;  // [chunk * cell1]
  int32_t *perm;              // [chunk * cell1]
  int32_t *status;            // [chunk * nelements]: 1 singular
  double *slpf;               // [nact * nions_total]
  int32_t *done;              // [nact]
};

// nltepop.cc:24-38 get_nlte_vector_index
DEVFN int nl_vindex(const Ctx &K, int e, int i, int l) {
  const int ui = uion(K, e, i);
  const int gs_index = K.T.ion_first_nlte[ui] - K.T.ion_first_nlte[uion(K, e, 0)] + i;
  const int nn = K.T.ion_nlevels_nlte[ui];
  return gs_index + ((l <= nn) ? l : (nn + 1));
}
// nltepop.cc:1543-1554 superlevel_boltzmann
DEVFN double nl_superlevel_boltzmann(const Ctx &K, const NlDev &N, int mgi, int ui, int l) {
  const int ul0 = K.T.ion_uniqueleveloffset[ui];
  const int sl = ul0 + K.T.ion_nlevels_nlte[ui] + 1;
  const double T_exc = K.R.exc_te ? (double)N.Te[mgi] : (double)N.TJ[mgi];
  return (double)K.T.level_stat_weight[ul0 + l] / (double)K.T.level_stat_weight[sl] *
         exp(-(K.T.level_epsilon[ul0 + l] - K.T.level_epsilon[sl]) / ARTIS_KB / T_exc);
}
// ltepop.cc:329-347 calculate_levelpop_lte
DEVFN double nl_levelpop_lte(const Ctx &K, const NlDev &N, int mgi, int e, int ui, int l) {
  const double nnground = nl_gpop(K, N, mgi, e, ui);
  if (l == 0) return nnground;
  const double T_exc = K.R.exc_te ? (double)N.Te[mgi] : (double)N.TJ[mgi];
  const double W = 1.;
  const int ul0 = K.T.ion_uniqueleveloffset[ui];
  return (nnground * W * (double)K.T.level_stat_weight[ul0 + l] / (double)K.T.level_stat_weight[ul0] *
          exp(-(K.T.level_epsilon[ul0 + l] - K.T.level_epsilon[ul0]) / ARTIS_KB / T_exc));
}
// nltepop.cc:832-850: the superlevel partition function of every (active cell, ion)
__global__ void k_nl_slpf(Ctx K, NlDev N, NlMat M, const int32_t *act, int nact) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int ni = K.T.nions_total;
  if (idx >= (int64_t)nact * ni) return;
  const int a = (int)(idx / ni), ui = (int)(idx % ni);
  const int mgi = act[a];
  const int nn = K.T.ion_nlevels_nlte[ui], nlevels = K.T.ion_nlevels[ui];
  double slpf = 0.;
  if (nlevels > nn + 1)
    for (int level = nn + 1; level < nlevels; level++) slpf += nl_superlevel_boltzmann(K, N, mgi, ui, level);
  M.slpf[idx] = slpf;
}
// s_renorm (nltepop.cc:852-865) of level l of ion ui
DEVFN double nl_s_renorm(const Ctx &K, const NlDev &N, const NlMat &M, int a, int mgi, int ui, int l) {
  if (l <= K.T.ion_nlevels_nlte[ui]) return 1.0;
  return nl_superlevel_boltzmann(K, N, mgi, ui, l) / M.slpf[(int64_t)a * K.T.nions_total + ui];
}

// The rate matrix of element e of active cell a, column c (nltepop.cc:421-628, 866-920): the column's entries of the
// five process matrices, each accumulated in the reference's order (the column of a level's index receives that
// level's terms; recombination into an upper-ion level precedes that level's own ionisation because the reference
// walks the ions upwards), then summed, the normalisation row set and the column scaled by its LTE population.
// Context K: the solver's state (pops, corrphot of active position a).
__global__ void k_nl_matrix(Ctx K, NlDev N, NlMat M, const int32_t *act, int a0, int nchunk) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)nchunk * M.cell1) return;
  const int al = (int)(idx / M.cell1), q = (int)(idx % M.cell1);
  const int a = a0 + al;
  const int mgi = act[a];
  const int e = M.col_e[q];
  const int D = M.el_D[e];
  const int c = q - M.el_off1[e];
  const int i = M.col_ion[q], l0 = M.col_l0[q], l1 = M.col_l1[q];
  const int ui0 = uion(K, e, 0), ui = ui0 + i;
  const int nions = K.T.elem_nions[e];
  const int64_t DD = (int64_t)D * D;
  double *Acol = M.A + (int64_t)al * M.cell2 + M.el_off2[e] + (int64_t)c * D;
  double *P = M.P + (int64_t)al * 5 * M.cell2 + 5 * M.el_off2[e] + (int64_t)c * D;
  double *P1 = P, *P2 = P + DD, *P3 = P + 2 * DD, *P4 = P + 3 * DD, *P5 = P + 4 * DD;
  for (int r = 0; r < D; r++) P1[r] = P2[r] = P3[r] = P4[r] = P5[r] = 0.;
  const double *pops = K.C.pops + (int64_t)a * K.T.nlevels_total;
  const double *corr = K.C.corrphot + (int64_t)a * K.T.ntargets_total;
  const float T_e = N.Te[mgi];
  const float nne = N.nne[mgi];
  const double t_mid = M.t_mid;
  const int ul0 = K.T.ion_uniqueleveloffset[ui];
  // bound-bound (nltepop.cc:421-505)
  for (int level = l0; level <= l1; level++) {
    const int ul = ul0 + level;
    const double sr = nl_s_renorm(K, N, M, a, mgi, ui, level);
    const double epsilon_level = K.T.level_epsilon[ul];
    const double statweight = K.T.level_stat_weight[ul];
    for (int k = 0; k < K.T.level_ndowntrans[ul]; k++) {
      const int li = K.T.downtrans_lineindex[K.T.level_downtrans_offset[ul] + k];
      const int lower = K.T.line_lower[li];
      const double epsilon_trans = epsilon_level - K.T.level_epsilon[ul0 + lower];
      const double R = rad_deexcitation_ratecoeff(K, pops, e, i, level, lower, epsilon_trans, li, t_mid) * sr;
      const double C = col_deexcitation_ratecoeff(K, T_e, nne, epsilon_trans, li, K.T.level_stat_weight[ul0 + lower],
                                                  statweight) * sr;
      const int lower_index = nl_vindex(K, e, i, lower);
      P1[c] -= R;
      P1[lower_index] += R;
      P2[c] -= C;
      P2[lower_index] += C;
    }
    for (int k = 0; k < K.T.level_nuptrans[ul]; k++) {
      const int li = K.T.uptrans_lineindex[K.T.level_uptrans_offset[ul] + k];
      const int upper = K.T.line_upper[li];
      const double epsilon_trans = K.T.level_epsilon[ul0 + upper] - epsilon_level;
      const double R = rad_excitation_ratecoeff(K, pops, mgi, e, i, level, upper, epsilon_trans, li, t_mid) * sr;
      const double C = col_excitation_ratecoeff(K, T_e, nne, li, epsilon_trans, statweight,
                                                K.T.level_stat_weight[ul0 + upper]) * sr;
      const int upper_index = nl_vindex(K, e, i, upper);
      P1[c] -= R;
      P1[upper_index] += R;
      P2[c] -= C;
      P2[upper_index] += C;
    }
  }
  // bound-free (nltepop.cc:507-562): recombination from this ion into the column (walking the lower ion), then the
  // column's own ionisation
  if (i > 0) {
    const int uil = ui - 1;
    const int nlev_lower = K.T.ion_nlevels[uil];
    const int maxrec = K.T.ion_maxrecombininglevel[ui];
    for (int level = 0; level < K.T.ion_ionisinglevels[uil]; level++) {
      for (int t = 0; t < get_nphixstargets(K, e, i - 1, level); t++) {
        const int upper = get_phixsupperlevel(K, e, i - 1, level, t);
        if (upper > maxrec || nl_vindex(K, e, i, upper) != c) continue;
        const double epsilon_trans = K.T.level_epsilon[ul0 + upper] - K.T.level_epsilon[K.T.ion_uniqueleveloffset[uil] + level];
        const double R_recomb = rad_recombination_ratecoeff(K, T_e, nne, e, i, upper, level);
        const double C_recomb = col_recombination_ratecoeff(K, mgi, e, i, upper, level, epsilon_trans);
        // D13: the lower ion's s_renorm at the upper level's number, 0 past its levels
        const double sr = (upper < nlev_lower) ? nl_s_renorm(K, N, M, a, mgi, uil, upper) : 0.;
        const int lower_index = nl_vindex(K, e, i - 1, level);
        P3[c] -= R_recomb * sr;
        P3[lower_index] += R_recomb * sr;
        P4[c] -= C_recomb * sr;
        P4[lower_index] += C_recomb * sr;
      }
    }
  }
  if (i < nions - 1) {
    for (int level = l0; level <= l1 && level < K.T.ion_ionisinglevels[ui]; level++) {
      const double sr = nl_s_renorm(K, N, M, a, mgi, ui, level);
      const double epsilon_current = K.T.level_epsilon[ul0 + level];
      const int slot0 = K.T.level_phixstargets_offset[ul0 + level];
      for (int t = 0; t < get_nphixstargets(K, e, i, level); t++) {
        const int upper = get_phixsupperlevel(K, e, i, level, t);
        const int upper_index = nl_vindex(K, e, i + 1, upper);
        const double epsilon_trans = epsilon(K, e, i + 1, upper) - epsilon_current;
        const double R_ionisation = corr[slot0 + t];
        const double C_ionisation = col_ionization_ratecoeff(K, T_e, nne, e, i, level, t, epsilon_trans);
        P3[c] -= R_ionisation * sr;
        P3[upper_index] += R_ionisation * sr;
        P4[c] -= C_ionisation * sr;
        P4[upper_index] += C_ionisation * sr;
      }
    }
    // non-thermal ionisation (nltepop.cc:564-591)
    if (K.R.nt_on) {
      const double Y_nt = N.ntY[(int64_t)mgi * K.T.nions_total + ui];
      for (int upperion = i + 1; upperion <= nt_ionisation_maxupperion(K, e, i); upperion++) {
        const double Y_nt_thisupperion = Y_nt * nt_ionization_upperion_probability(K, mgi, e, i, upperion, false);
        if (Y_nt_thisupperion > 0.) {
          const int upper_groundstate_index = nl_vindex(K, e, upperion, 0);
          for (int level = l0; level <= l1; level++) {
            const double sr = nl_s_renorm(K, N, M, a, mgi, ui, level);
            P5[c] -= Y_nt_thisupperion * sr;
            P5[upper_groundstate_index] += Y_nt_thisupperion * sr;
          }
        }
      }
    }
  }
  // nltepop.cc:593-628 nltepop_matrix_normalise: LTE population of the column's level (or of the superlevel's)
  double norm = nl_levelpop_lte(K, N, mgi, e, ui, l0);
  if (l0 != 0 && l0 > K.T.ion_nlevels_nlte[ui])
    for (int dl = l0 + 1; dl < K.T.ion_nlevels[ui]; dl++) norm += nl_levelpop_lte(K, N, mgi, e, ui, dl);
  for (int r = 0; r < D; r++) {
    double v = ((((0. + P1[r]) + P2[r]) + P3[r]) + P4[r]) + P5[r];
    if (r == 0) v = 1.0;
    Acol[r] = v * norm;
  }
  const int64_t vo = (int64_t)al * M.cell1 + M.el_off1[e] + c;
  M.norm[vo] = norm;
  M.b[vo] = (c == 0) ? nl_elem_numberdens(K, N, mgi, e) : 0.;
}

// nltepop.cc:656-796 nltepop_matrix_solve for one (cell, element) per workgroup: LU with partial pivoting (D11),
// x = LU^-1 b, ten refinement passes keeping the smallest max-norm residual (stop below 1e-40), populations scaled
// back by the normalisation; status 1: singular
#define NL_LU_WG 256
__global__ __launch_bounds__(NL_LU_WG) void k_nl_lu(Ctx K, NlMat M, int nchunk) {
  __shared__ double s_v[NL_LU_WG];
  __shared__ int s_i[NL_LU_WG];
  __shared__ int s_flag;
  __shared__ double s_err;
  const int ne = K.T.nelements;
  const int al = blockIdx.x / ne, e = blockIdx.x % ne;
  if (al >= nchunk) return;
  const int D = M.el_D[e];
  if (D == 0) return;
  const int tid = threadIdx.x;
  const int64_t o2 = (int64_t)al * M.cell2 + M.el_off2[e];
  const int64_t o1 = (int64_t)al * M.cell1 + M.el_off1[e];
  const double *A = M.A + o2;
  double *LU = M.LU + o2;
  const double *b = M.b + o1, *norm = M.norm + o1;
  double *xv = M.xv + o1, *best = M.best + o1, *work = M.work + o1, *res = M.res + o1, *pv = M.pv + o1;
  int32_t *perm = M.perm + o1;
  for (int64_t q = tid; q < (int64_t)D * D; q += NL_LU_WG) LU[q] = A[q];
  for (int r = tid; r < D; r += NL_LU_WG) perm[r] = r;
  __syncthreads();
  for (int j = 0; j < D - 1; j++) {
    double amax = -1.;
    int imax = D;
    for (int r = j + tid; r < D; r += NL_LU_WG) {
      const double v = fabs(LU[(int64_t)j * D + r]);
      if (v > amax) {
        amax = v;
        imax = r;
      }
    }
    s_v[tid] = amax;
    s_i[tid] = imax;
    __syncthreads();
    for (int w = NL_LU_WG / 2; w > 0; w >>= 1) {
      if (tid < w) {
        const double v = s_v[tid + w];
        const int iv = s_i[tid + w];
        if (v > s_v[tid] || (v == s_v[tid] && iv < s_i[tid])) {
          s_v[tid] = v;
          s_i[tid] = iv;
        }
      }
      __syncthreads();
    }
    int i_pivot = s_i[0];
    // the sequential scan keeps row j unless a later |a_ij| is strictly larger (NaN never is)
    const double ajj_abs = fabs(LU[(int64_t)j * D + j]);
    if (!(s_v[0] > ajj_abs) || i_pivot >= D) i_pivot = j;
    __syncthreads();
    if (i_pivot != j) {
      for (int k = tid; k < D; k += NL_LU_WG) {
        const double t = LU[(int64_t)k * D + j];
        LU[(int64_t)k * D + j] = LU[(int64_t)k * D + i_pivot];
        LU[(int64_t)k * D + i_pivot] = t;
      }
      if (tid == 0) {
        const int t = perm[j];
        perm[j] = perm[i_pivot];
        perm[i_pivot] = t;
      }
    }
    __syncthreads();
    const double ajj = LU[(int64_t)j * D + j];
    if (ajj != 0.0) {
      for (int r = j + 1 + tid; r < D; r += NL_LU_WG) LU[(int64_t)j * D + r] = LU[(int64_t)j * D + r] / ajj;
      __syncthreads();
      const int m = D - j - 1;
      for (int64_t q = tid; q < (int64_t)m * m; q += NL_LU_WG) {
        const int r = j + 1 + (int)(q % m), k = j + 1 + (int)(q / m);
        LU[(int64_t)k * D + r] = LU[(int64_t)k * D + r] - LU[(int64_t)j * D + r] * LU[(int64_t)k * D + j];
      }
    }
    __syncthreads();
  }
  if (tid == 0) {
    s_flag = 0;
    for (int r = 0; r < D; r++)
      if (LU[(int64_t)r * D + r] == 0) s_flag = 1;
    M.status[al * ne + e] = s_flag;
  }
  __syncthreads();
  if (s_flag) return;
  // gsl_linalg_LU_svx on v: permute (v'_i = v_{p_i}), unit-lower then upper, both column-oriented
  auto svx = [&](double *v) {
    for (int r = tid; r < D; r += NL_LU_WG) res[r] = v[r];
    __syncthreads();
    for (int r = tid; r < D; r += NL_LU_WG) v[r] = res[perm[r]];
    __syncthreads();
    for (int j = 0; j < D; j++) {
      const double xj = v[j];
      for (int r = j + 1 + tid; r < D; r += NL_LU_WG) v[r] -= LU[(int64_t)j * D + r] * xj;
      __syncthreads();
    }
    for (int j = D - 1; j >= 0; j--) {
      if (tid == 0) v[j] = v[j] / LU[(int64_t)j * D + j];
      __syncthreads();
      const double xj = v[j];
      for (int r = tid; r < j; r += NL_LU_WG) v[r] -= LU[(int64_t)j * D + r] * xj;
      __syncthreads();
    }
  };
  auto residual = [&](const double *x, double *out) {  // A x - b, row-serial
    for (int r = tid; r < D; r += NL_LU_WG) {
      double temp = 0.;
      for (int j = 0; j < D; j++) temp += x[j] * A[(int64_t)j * D + r];
      out[r] = -b[r] + temp;
    }
    __syncthreads();
  };
  for (int r = tid; r < D; r += NL_LU_WG) xv[r] = b[r];
  __syncthreads();
  svx(xv);
  if (tid == 0) s_err = -1.;
  __syncthreads();
  for (int iteration = 0; iteration < 10; iteration++) {
    if (iteration > 0) {
      residual(xv, work);
      svx(work);
      for (int r = tid; r < D; r += NL_LU_WG) xv[r] += -1.0 * work[r];
      __syncthreads();
    }
    residual(xv, work);
    if (tid == 0) {
      int imax = 0;
      double amax = -1.;
      for (int r = 0; r < D; r++)
        if (fabs(work[r]) > amax) {
          amax = fabs(work[r]);
          imax = r;
        }
      const double error = fabs(work[imax]);
      s_flag = (error < s_err || s_err < 0.) ? 1 : 0;
      if (s_flag) s_err = error;
      if (error < 1e-40) s_flag |= 2;
    }
    __syncthreads();
    const int fl = s_flag;
    if (fl & 1)
      for (int r = tid; r < D; r += NL_LU_WG) best[r] = xv[r];
    __syncthreads();
    if (fl & 2) break;
  }
  for (int r = tid; r < D; r += NL_LU_WG) {
    double v = best[r] * norm[r];
    if (v < 0.0) v = norm[r];
    pv[r] = v;
  }
}

// nltepop.cc:376-389 set_element_pops_lte: no NLTE solution for the element
DEVFN void nl_reset_element(const Ctx &K, const NlDev &N, int mgi, int e) {
  double *row = N.nlte + (int64_t)mgi * K.T.total_nlte_levels;
  for (int i = 0; i < K.T.elem_nions[e]; i++) {
    const int ui = uion(K, e, i);
    const int nlte_start = K.T.ion_first_nlte[ui];
    const int nn = K.T.ion_nlevels_nlte[ui];
    for (int level = 1; level < nn; level++) row[nlte_start + level - 1] = -1.0;
    if (K.T.ion_nlevels[ui] > nn + 1) row[nlte_start + nn] = -1.0;
  }
}
// nltepop.cc:1040-1113 the solved populations into the cell state; then update_grid.cc:845-853 precalculate_partfuncts,
// calculate_electron_densities and the convergence test of solve_Te_nltepops.  One workitem per active cell of the
// chunk.
__global__ void k_nl_store(const Ctx *__restrict__ Kp, const TeDev *__restrict__ Dp, NlDev N, NlMat M,
                           const int32_t *act, int a0, int nchunk) {
  const Ctx &K = *Kp;
  const TeDev &D = *Dp;
  const int al = blockIdx.x * blockDim.x + threadIdx.x;
  if (al >= nchunk) return;
  const int a = a0 + al;
  const int mgi = act[a];
  const int ne = K.T.nelements, ni = K.T.nions_total;
  for (int e = 0; e < ne; e++) {
    const int nions = K.T.elem_nions[e];
    if (nions <= 0) continue;
    if (N.abund[(int64_t)mgi * ne + e] <= 0.) {
      nl_reset_element(K, N, mgi, e);
      continue;
    }
    if (M.status[al * ne + e]) {
      nl_reset_element(K, N, mgi, e);
      continue;
    }
    const int Dm = M.el_D[e];
    const double *pv = M.pv + (int64_t)al * M.cell1 + M.el_off1[e];
    bool bad = false;
    for (int k = 0; k < Dm; k++)
      if (!isfinite(pv[k]) || !(pv[k] >= 0.)) bad = true;
    if (bad) {
      nl_fail(N, mgi, NLF_POPS);
      return;
    }
    double *row = N.nlte + (int64_t)mgi * K.T.total_nlte_levels;
    const double rho = N.rho[mgi];
    for (int i = 0; i < nions; i++) {
      const int ui = uion(K, e, i);
      const int nn = K.T.ion_nlevels_nlte[ui];
      const int index_gs = nl_vindex(K, e, i, 0);
      const int nlte_start = K.T.ion_first_nlte[ui];
      for (int level = 1; level <= nn; level++) row[nlte_start + level - 1] = pv[nl_vindex(K, e, i, level)] / rho;
      if (K.T.ion_nlevels[ui] > nn + 1)
        row[nlte_start + nn] = (pv[nl_vindex(K, e, i, nn + 1)] / rho / M.slpf[(int64_t)a * ni + ui]);
      N.gp[(int64_t)mgi * ni + ui] = pv[index_gs];
    }
    double elem_pop_matrix = 0.;
    for (int k = 0; k < Dm; k++) elem_pop_matrix += fabs(pv[k]);
    const double elem_pop_abundance = nl_elem_numberdens(K, N, mgi, e);
    const double elem_pop_error_percent = fabs((elem_pop_abundance / elem_pop_matrix) - 1) * 100;
    if (elem_pop_error_percent > 1.0) nl_reset_element(K, N, mgi, e);
  }
  const double nne_prev = N.nne[mgi];
  TeState s;
  s.k = a;
  s.mgi = mgi;
  s.Te = N.Te[mgi];
  s.g = 1;
  s.sub = 0;
  s.lane0 = 0;
  s.phi = nullptr;
  te_precalculate_partfuncts(K, D, s);
  te_electron_densities(K, D, s);
  const double fracdiff_nne = fabs((N.nne[mgi] / nne_prev) - 1);
  const double fracdiff_T_e = fabs((N.Te[mgi] / N.prevTe[mgi]) - 1);
  M.done[a] = (fracdiff_nne <= 0.04 && fracdiff_T_e <= 0.04) ? 1 : 0;
}
