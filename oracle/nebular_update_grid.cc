// nebular_update_grid.cc -- included at the end of oracle.cc (it uses that file's anonymous-namespace helpers).
//
// TEST INFRASTRUCTURE ONLY (see oracle.cc's header): the CPU checker of artis_gpu_update_grid_nlte, update_grid for the
// nebular options (artisoptions_nltenebular.h) restated serially from the reference, one model cell per OpenMP
// iteration.  Parity unpinned like the rest of the oracle; its own pins are in tests/test_nebular_update_grid.py
// (LU against LAPACK through numpy, Planck integrals against closed forms, the Spencer-Fano system against its
// residual and the degradation-energy sum, column conservation of the NLTE rate matrix).
//
// Deviations (identical in the engine):
//   D10 sfmatrix_add_ionization's second integral (nonthermal.cc:2405-2419) starts at get_energyindex_ev_lteq(2E + I),
//       which can lie below the shell's xsstartindex, where the reference reads prefactors[] / int_eps_upper[] that
//       it never set (stack arrays, nonthermal.cc:2365-2372).  Those terms are skipped here: the cross section they
//       would multiply is zero below xsstartindex.
//   D11 GSL's LU (version unpinned; GSL 2.7.1 in the reference CI, whose LU_decomp is a recursive blocked variant) is
//       restated as the unblocked right-looking LU with partial pivoting of GSL <= 2.6 (linalg/lu.c), and the upper
//       triangular solve is column-oriented (x_j final, then every x_i, i < j, updated) instead of cblas dtrsv's
//       row-oriented dot products (the lower unit-triangular solve keeps dtrsv's order).  Every partial-pivoting LU
//       agrees to rounding; tests/ pin this one against LAPACK.
//   D12 calculate_frac_heating (nonthermal.cc:1102-1150) is not evaluated: analyse_sf_solution overwrites its result
//       with 1 - frac_excitation - frac_ionization (nonthermal.cc:2258-2268); it only prints it.  The degradation
//       sum is checked in tests/ instead (oracle_sf_frac_heating).
namespace {

constexpr int kNtMaxAuger = ARTIS_NT_MAX_AUGER;
constexpr double kMinIonFraction = 1.e-8;        // nonthermal.cc:61
constexpr double kANaughtSquared = 2.800285203e-17;  // nonthermal.cc:67
constexpr int kMNtShells = 10, kMaxZBinding = 30;    // nonthermal.cc:70-73
constexpr int kNtExcMaxLower = 5, kNtExcMaxUpper = 250;  // artisoptions_nltenebular.h:169-170

// the mutable grid state one cell's solution writes (grid::modelgrid[mgi], radfield, nt_solution); Ctx::cs points
// at these arrays
struct NlteGrid {
  std::vector<float> Te, TR, W, TJ, nne, nnetot, gp, pf, binTR, binW, bfrate;
  std::vector<double> nlte_pops, ntY;
  std::vector<float> nt_prob, nt_ionen;
};

// the Spencer-Fano energy grid (nonthermal.cc:555-618, SF_USE_LOG_E_INCREMENT false)
struct SfGrid {
  int n = 0;
  double emin = 0., emax = 0., delta_e = 0., E_init_ev = 0.;
  std::vector<double> envec, logenvec, sourcevec;
};

struct NlteRun {
  const artis_nlte_params *p;
  const artis_nt_shells *nt;
  const artis_nlte_cells *in;
  NlteGrid *g;
  SfGrid sf;
};

inline size_t nix(const Ctx &c, int mgi, int e, int i) { return (size_t)mgi * c.at->nions_total + uion(c, e, i); }
inline float &nl_gp(const Ctx &c, const NlteRun &r, int mgi, int e, int i) { return r.g->gp[nix(c, mgi, e, i)]; }
inline float &nl_pf(const Ctx &c, const NlteRun &r, int mgi, int e, int i) { return r.g->pf[nix(c, mgi, e, i)]; }
// grid.cc:231-236
inline double nl_elem_numberdens(const Ctx &c, const NlteRun &r, int mgi, int e) {
  const size_t k = (size_t)mgi * c.at->nelements + e;
  return r.in->elem_abundance[k] / r.in->elem_meanweight[k] * (double)r.in->rho[mgi];
}
// atomic.cc:58-66 get_nntot
double nl_get_nntot(const Ctx &c, const NlteRun &r, int mgi) {
  double nntot = 0.;
  for (int e = 0; e < c.at->nelements; e++) nntot += nl_elem_numberdens(c, r, mgi, e);
  return nntot;
}

// ltepop.cc:488-537 calculate_partfunct (NLTE-aware through calculate_levelpop_nominpop)
double nl_calculate_partfunct(const Ctx &c, const NlteRun &r, int mgi, int e, int i) {
  int initial = 0;
  double pop_store = 0.;
  if (get_groundlevelpop(c, mgi, e, i) < c.minpop) {
    pop_store = get_groundlevelpop(c, mgi, e, i);
    initial = 1;
    nl_gp(c, r, mgi, e, i) = 1.0;
  }
  double U = 1.;
  const int nlevels = get_nlevels(c, e, i);
  const double groundpop = get_groundlevelpop(c, mgi, e, i);
  for (int level = 1; level < nlevels; level++) {
    bool skipminpop;
    const double nn = calculate_levelpop_nominpop(c, mgi, e, i, level, &skipminpop) / groundpop;
    U += nn;
  }
  U *= stat_weight(c, e, i, 0);
  if (initial == 1) nl_gp(c, r, mgi, e, i) = pop_store;
  return U;
}
// update_grid.cc:23-38
void nl_precalculate_partfuncts(const Ctx &c, const NlteRun &r, int mgi) {
  for (int e = 0; e < c.at->nelements; e++)
    for (int i = 0; i < get_nions(c, e); i++) nl_pf(c, r, mgi, e, i) = nl_calculate_partfunct(c, r, mgi, e, i);
}
// update_grid.cc:1660-1685 calculate_electron_densities: returns nne_tot
double nl_calculate_electron_densities(const Ctx &c, const NlteRun &r, int mgi) {
  double nne_tot = 0.;
  float nne = 0.;
  for (int e = 0; e < c.at->nelements; e++) {
    const double nnelement = nl_elem_numberdens(c, r, mgi, e);
    nne_tot += nnelement * c.at->elem_anumber[e];
    if (nnelement > 0) {
      for (int i = 0; i < get_nions(c, e); i++) nne += (get_ionstage(c, e, i) - 1) * ionstagepop(c, mgi, e, i);
    }
  }
  r.g->nne[mgi] = nne;
  r.g->nnetot[mgi] = nne_tot;
  return nne_tot;
}

// update_grid.cc:1427-1658 calculate_populations in the LTE branch (use_lte_ratio: LTE phi, every ion up to the top)
int nl_calculate_populations_lte(const Ctx &c, const NlteRun &r, int mgi) {
  const int nel = c.at->nelements;
  double nne_hi = r.in->rho[mgi] / ARTIS_MH;
  std::vector<int> upp(nel, 0);
  auto phi = [&](int e, int i) {  // ltepop.cc:152-158
    const float T_e = r.g->Te[mgi];
    const double ionpot = epsilon(c, e, i + 1, 0) - epsilon(c, e, i, 0);
    const double partfunct_ratio = nl_pf(c, r, mgi, e, i) / nl_pf(c, r, mgi, e, i + 1);
    return partfunct_ratio * ARTIS_SAHACONST * pow(T_e, -1.5) * exp(ionpot / ARTIS_KB / T_e);
  };
  auto ionfractions = [&](int e, double nne, double *fr, int uppermost_ion) {  // ltepop.cc:61-95
    double nnionfactor[64];
    nnionfactor[uppermost_ion] = 1;
    double denominator = 1.;
    for (int ion = uppermost_ion - 1; ion >= 0; ion--) {
      nnionfactor[ion] = nnionfactor[ion + 1] * nne * phi(e, ion);
      denominator += nnionfactor[ion];
    }
    for (int ion = 0; ion <= uppermost_ion; ion++) {
      fr[ion] = nnionfactor[ion] / denominator;
      if (!std::isfinite(fr[ion])) fr[ion] = 0;
    }
  };
  int only_neutral_ions = 0, nelements_in_cell = 0;
  for (int e = 0; e < nel; e++) {
    const int nions = get_nions(c, e);
    upp[e] = nions - 1;
    if (r.in->elem_abundance[(size_t)mgi * nel + e] > 0) {
      const int uppermost_ion0 = nions - 1;
      double factor = 1.;
      int ion;
      for (ion = 0; ion < uppermost_ion0; ion++) {
        factor *= nne_hi * phi(e, ion);
        if (!std::isfinite(factor)) break;
      }
      upp[e] = ion;
      if (ion == 0) only_neutral_ions++;
      nelements_in_cell++;
    }
  }
  float nne = 0.;
  double nne_tot = 0.;
  if (only_neutral_ions == nelements_in_cell) {
    for (int e = 0; e < nel; e++) {
      const double nnelement = nl_elem_numberdens(c, r, mgi, e);
      nne_tot += nnelement * c.at->elem_anumber[e];
      for (int ion = 0; ion < get_nions(c, e); ion++) {
        const double nnion = (ion == 0) ? nnelement : (nnelement > 0. ? c.minpop : 0.);
        nne += nnion * (get_ionstage(c, e, ion) - 1);
        nl_gp(c, r, mgi, e, ion) = (nnion * stat_weight(c, e, ion, 0) / nl_pf(c, r, mgi, e, ion));
      }
    }
    if (nne < c.minpop) nne = c.minpop;
    r.g->nne[mgi] = nne;
  } else {
    auto f = [&](double x) {  // ltepop.cc:20-59
      const double rho = r.in->rho[mgi];
      double outersum = 0.;
      for (int e = 0; e < nel; e++) {
        const float abundance = r.in->elem_abundance[(size_t)mgi * nel + e];
        if (abundance > 0 && get_nions(c, e) > 0) {
          const double elem_mw = r.in->elem_meanweight[(size_t)mgi * nel + e];
          double fr[64];
          ionfractions(e, x, fr, upp[e]);
          double innersum = 0.;
          for (int ion = 0; ion <= upp[e]; ion++) innersum += (get_ionstage(c, e, ion) - 1) * fr[ion];
          outersum += abundance / elem_mw * innersum;
        }
      }
      return rho * outersum - x;
    };
    double nne_lo = 0.;
    GslBrent s;
    if (gsl_brent_set(s, f, nne_lo, nne_hi) != 0) return -1;
    int iter = 0, status;
    do {
      iter++;
      if (gsl_brent_iterate(s, f) != 0) return -1;
      nne = s.root;
      nne_lo = s.x_lower;
      nne_hi = s.x_upper;
      status = gsl_test_interval(nne_lo, nne_hi, 0, 1e-3);
    } while (status == 1 && iter < 100);
    if (nne < c.minpop) nne = c.minpop;
    r.g->nne[mgi] = nne;
    for (int e = 0; e < nel; e++) {
      const double nnelement = nl_elem_numberdens(c, r, mgi, e);
      nne_tot += nnelement * c.at->elem_anumber[e];
      double fr[64];
      if (nnelement > 0) ionfractions(e, nne, fr, upp[e]);
      for (int ion = 0; ion < get_nions(c, e); ion++) {
        double nnion;
        if (ion <= upp[e]) {
          if (nnelement > 0) {
            nnion = nnelement * fr[ion];
            if (nnion < c.minpop) nnion = c.minpop;
          } else {
            nnion = 0.;
          }
        } else {
          nnion = c.minpop;
        }
        nl_gp(c, r, mgi, e, ion) = (nnion * stat_weight(c, e, ion, 0) / nl_pf(c, r, mgi, e, ion));
      }
    }
  }
  r.g->nnetot[mgi] = nne_tot;
  return 0;
}

// ---------------------------------------------------------------------------------- radiation field fit
// radfield.cc:945-954 gsl_integrand_planck, 957-979 planck_integral (qag GK61, epsrel 1e-10; a failed integral is 0)
double nl_planck_integral(double T_R, double nu_lower, double nu_upper, bool times_nu) {
  auto f = [&](double nu) {
    double integrand = ARTIS_TWOHOVERCLIGHTSQUARED * pow(nu, 3) / (expm1(ARTIS_HOVERKB * nu / T_R));
    if (times_nu) integrand *= nu;
    return integrand;
  };
  static thread_local GslWorkspace ws(kGslWsSize);
  double integral = 0., error = 0.;
  const int status = gsl_qag61(f, nu_lower, nu_upper, 0., 1e-10, kGslWsSize, ws, &integral, &error);
  if (status != 0) integral = 0.;
  return integral;
}
inline double bin_nu_lower(const Ctx &c, int b) {
  return b > 0 ? c.at->radfield_nu_upper[b - 1] : c.at->radfield_nu_lower_first;
}
// radfield.cc:1020-1066 delta_nu_bar, 1070-1133 find_T_R; *fail on GSL's default error handler (a non-finite
// function value inside the Brent iteration aborts the reference)
float nl_find_T_R(const Ctx &c, const NlteRun &r, double nu_bar_estimator, int b, int *fail) {
  const double nu_lower = bin_nu_lower(c, b), nu_upper = c.at->radfield_nu_upper[b];
  auto delta_nu_bar = [&](double T_R) {
    const double nu_times_planck = nl_planck_integral(T_R, nu_lower, nu_upper, true);
    const double planck = nl_planck_integral(T_R, nu_lower, nu_upper, false);
    return nu_times_planck / planck - nu_bar_estimator;
  };
  const double T_R_min = r.p->T_R_min, T_R_max = r.p->T_R_max;
  double delta_nu_bar_min = delta_nu_bar(T_R_min);
  double delta_nu_bar_max = delta_nu_bar(T_R_max);
  if (!std::isfinite(delta_nu_bar_min) || !std::isfinite(delta_nu_bar_max)) delta_nu_bar_max = delta_nu_bar_min = -1;
  double T_R = 0.;
  if (delta_nu_bar_min * delta_nu_bar_max < 0) {
    GslBrent s;
    if (gsl_brent_set(s, delta_nu_bar, T_R_min, T_R_max) != 0) {
      *fail = 1;
      return 0.f;
    }
    int iteration_num = 0, status;
    do {
      iteration_num++;
      if (gsl_brent_iterate(s, delta_nu_bar) != 0) {
        *fail = 1;
        return 0.f;
      }
      T_R = s.root;
      status = gsl_test_interval(s.x_lower, s.x_upper, 0., 1e-4);
    } while (status == 1 && iteration_num < 100);
  } else if (delta_nu_bar_max < 0) {
    T_R = T_R_max;
  } else {
    T_R = T_R_min;
  }
  return T_R;
}
// radfield.cc:1136-1175 set_params_fullspec, 1177-1291 fit_parameters (J and nuJ already normalised)
void nl_fit_parameters(const Ctx &c, const NlteRun &r, int mgi, double J, double nuJ, double J_normfactor, int *fail) {
  const double nubar = nuJ / J;
  if (std::isfinite(nubar) && nubar != 0.) {
    float T_J = pow(J * ARTIS_PI / ARTIS_STEBO, 1 / 4.);
    if (T_J > r.p->T_max)
      T_J = r.p->T_max;
    else if (T_J < r.p->T_min)
      T_J = r.p->T_min;
    r.g->TJ[mgi] = T_J;
    float T_R = ARTIS_H * nubar / ARTIS_KB / 3.832229494;
    if (T_R > r.p->T_max)
      T_R = r.p->T_max;
    else if (T_R < r.p->T_min)
      T_R = r.p->T_min;
    r.g->TR[mgi] = T_R;
    r.g->W[mgi] = J * ARTIS_PI / ARTIS_STEBO / pow(T_R, 4);
  }
  const int nb = c.at->radfield_nbins;
  for (int b = 0; b < nb; b++) {
    const size_t mb = (size_t)mgi * nb + b;
    const double nu_lower = bin_nu_lower(c, b), nu_upper = c.at->radfield_nu_upper[b];
    const double J_bin = r.in->bin_J_raw[mb] * J_normfactor;
    float T_R_bin = -1.0;
    double W_bin = -1.0;
    if (r.in->bin_contribcount[mb] > 0) {
      const double nu_bar = (r.in->bin_nuJ_raw[mb] * J_normfactor) / J_bin;  // get_bin_nu_bar
      T_R_bin = nl_find_T_R(c, r, nu_bar, b, fail);
      if (b == nb - 1) T_R_bin = r.g->Te[mgi];
      double planck_integral_result = nl_planck_integral(T_R_bin, nu_lower, nu_upper, false);
      W_bin = J_bin / planck_integral_result;
      if (W_bin > 1e4) {
        planck_integral_result = nl_planck_integral(r.p->T_R_max, nu_lower, nu_upper, false);
        W_bin = J_bin / planck_integral_result;
        if (W_bin > 1e4) {
          T_R_bin = -99.0;
          W_bin = 0.;
        } else {
          T_R_bin = r.p->T_R_max;
        }
      }
    } else {
      T_R_bin = 0.;
      W_bin = 0.;
    }
    r.g->binTR[mb] = T_R_bin;
    r.g->binW[mb] = W_bin;
  }
}

// thermalbalance.cc:60-132 calculate_bfheatingcoeff (NO_LUT_BFHEATING), 141-187 calculate_bfheatingcoeffs
double nl_calculate_bfheatingcoeff(const Ctx &c, const NlteRun &r, int e, int i, int l, int t, int mgi) {
  const double E_threshold = get_phixs_threshold(c, e, i, l, t);
  const double nu_threshold = ARTIS_ONEOVERH * E_threshold;
  const double nu_max_phixs = nu_threshold * c.at->last_phixs_nuovernuedge;
  const float T_R = r.g->TR[mgi];
  const float *xs = level_photoion_xs(c, e, i, l);
  auto integrand = [&](double nu) {
    const float sigma_bf = (float)photoionization_crosssection_fromtable(c, xs, nu_threshold, nu);
    return sigma_bf * (1 - nu_threshold / nu) * radfield(c, nu, mgi) * (1 - exp(-ARTIS_HOVERKB * nu / T_R));
  };
  static thread_local GslWorkspace ws(kGslWsSize);
  double bfheating = 0., error = 0.;
  gsl_qag61(integrand, nu_threshold, nu_max_phixs, 0., 1e-3, kGslWsSize, ws, &bfheating, &error);
  bfheating *= ARTIS_FOURPI * get_phixsprobability(c, e, i, l, t);
  return bfheating;
}
int nl_calculate_bfheatingcoeffs(const Ctx &c, const NlteRun &r, int mgi, std::vector<double> &coeff) {
  const double minelfrac = 0.01;
  coeff.assign(c.at->nlevels_total, 0.);
  for (int e = 0; e < c.at->nelements; e++)
    for (int i = 0; i < get_nions(c, e); i++)
      for (int l = 0; l < get_nlevels(c, e, i); l++) {
        double bfheatingcoeff = 0.;
        if (r.in->elem_abundance[(size_t)mgi * c.at->nelements + e] > minelfrac) {
          for (int t = 0; t < get_nphixstargets(c, e, i, l); t++)
            bfheatingcoeff += nl_calculate_bfheatingcoeff(c, r, e, i, l, t, mgi);
          if (!std::isfinite(bfheatingcoeff)) return -1;  // assert_always (thermalbalance.cc:171)
        }
        coeff[ulev(c, e, i, l)] = bfheatingcoeff;
      }
  return 0;
}

// ------------------------------------------------------------------------------------------- Spencer-Fano
void sf_setup(SfGrid &s, const artis_nt_shells *nt) {
  s.n = nt->sfpts;
  s.emin = nt->sf_emin;
  s.emax = nt->sf_emax;
  s.delta_e = (s.emax - s.emin) / (s.n - 1);  // nonthermal.cc:111
  s.envec.assign(s.n, 0.);
  s.logenvec.assign(s.n, 0.);
  s.sourcevec.assign(s.n, 0.);
  const int source_spread_pts = (int)ceil(s.n * 0.03333);
  const double source_spread_en = source_spread_pts * s.delta_e;
  const int sourcelowerindex = s.n - source_spread_pts;
  for (int k = 0; k < s.n; k++) {
    const double energy_ev = s.emin + k * s.delta_e;
    s.envec[k] = energy_ev;
    s.logenvec[k] = log(energy_ev);
    s.sourcevec[k] = (k < sourcelowerindex) ? 0. : 1. / source_spread_en;
  }
  // E_init_ev = integral of E S(E) dE (gsl_vector_scale, gsl_vector_mul, gsl_blas_dasum)
  double E = 0.;
  for (int k = 0; k < s.n; k++) E += fabs((s.sourcevec[k] * s.delta_e) * s.envec[k]);
  s.E_init_ev = E;
}
// nonthermal.cc:757-789
inline int sf_lteq(const SfGrid &s, double energy_ev) {
  const int index = (int)floor((energy_ev - s.emin) / s.delta_e);
  return index < 0 ? 0 : (index > s.n - 1 ? s.n - 1 : index);
}
inline int sf_gteq(const SfGrid &s, double energy_ev) {
  const int index = (int)ceil((energy_ev - s.emin) / s.delta_e);
  return index < 0 ? 0 : (index > s.n - 1 ? s.n - 1 : index);
}
// nonthermal.cc:820-840 electron_loss_rate [erg / cm]
double sf_electron_loss_rate(double energy, double nne) {
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
// nonthermal.cc:872-929 get_xs_excitation_vector; -1: no cross section
int sf_xs_excitation_vector(const Ctx &c, const SfGrid &s, double *xs, int li, double statweight_lower,
                            double epsilon_trans) {
  const double coll_str = c.at->line_coll_str[li];
  if (coll_str >= 0) {
    const double constantfactor = pow(ARTIS_H_IONPOT, 2) / statweight_lower * coll_str * ARTIS_PI * kANaughtSquared;
    const int en_startindex = sf_gteq(s, epsilon_trans / ARTIS_EV);
    for (int j = 0; j < en_startindex; j++) xs[j] = 0.;
    for (int j = en_startindex; j < s.n; j++) {
      const double energy = s.envec[j] * ARTIS_EV;
      xs[j] = constantfactor * pow(energy, -2);
    }
    return en_startindex;
  }
  if (!c.at->line_forbidden[li]) {
    const double fij = c.at->line_osc_strength[li];
    const double A = 0.28, B = 0.15;
    const double prefactor = 45.585750051;
    const double epsilon_trans_ev = epsilon_trans / ARTIS_EV;
    const double constantfactor =
        epsilon_trans_ev * prefactor * kANaughtSquared * pow(ARTIS_H_IONPOT / epsilon_trans, 2) * fij;
    const int en_startindex = sf_gteq(s, epsilon_trans_ev);
    for (int j = 0; j < en_startindex; j++) xs[j] = 0.;
    for (int j = en_startindex; j < s.n; j++) {
      const double logU = s.logenvec[j] - log(epsilon_trans_ev);
      const double g_bar = A * logU + B;
      xs[j] = constantfactor * g_bar / s.envec[j];
    }
    return en_startindex;
  }
  return -1;
}
// nonthermal.cc:952-976 get_xs_ionization_vector
int sf_xs_ionization_vector(const SfGrid &s, const artis_nt_shells *nt, int k, double *xs) {
  const double ionpot_ev = nt->ionpot_ev[k];
  const int startindex = sf_gteq(s, ionpot_ev);
  for (int i = 0; i < startindex; i++) xs[i] = 0.;
  const double A = nt->A[k], B = nt->B[k], C = nt->C[k], D = nt->D[k];
  for (int i = startindex; i < s.n; i++) {
    const double u = s.envec[i] / ionpot_ev;
    xs[i] = 1e-14 * (A * (1 - 1 / u) + B * pow((1 - 1 / u), 2) + C * log(u) + D * log(u) / u) / (u * pow(ionpot_ev, 2));
  }
  return startindex;
}
// nonthermal.cc:994-1007
inline double sf_get_J(int Z, int ionstage, double ionpot_ev) {
  if (ionstage == 1) {
    if (Z == 2) return 15.8;
    if (Z == 10) return 24.2;
    if (Z == 18) return 10.0;
  }
  return 0.6 * ionpot_ev;
}
inline bool shell_matches(const artis_nt_shells *nt, int k, int Z, int ionstage) {
  return nt->Z[k] == Z && nt->nelec[k] == Z - ionstage + 1;
}
// nonthermal.cc:1193-1309 get_mean_binding_energy; -1 on the reference's abort paths
double sf_mean_binding_energy(const Ctx &c, const artis_nt_shells *nt, int e, int i, int *fail) {
  int q[kMNtShells];
  double total;
  const int ioncharge = get_ionstage(c, e, i) - 1;
  const int Zel = c.at->elem_anumber[e];
  const int nbound = Zel - ioncharge;
  if (nbound > 0) {
    for (int k = 0; k < kMNtShells; k++) q[k] = 0;
    for (int electron_loop = 0; electron_loop < nbound; electron_loop++) {
      if (q[0] < 2)
        q[0]++;
      else if (q[1] < 2)
        q[1]++;
      else if (q[2] < 2)
        q[2]++;
      else if (q[3] < 4)
        q[3]++;
      else if (q[4] < 2)
        q[4]++;
      else if (q[5] < 2)
        q[5]++;
      else if (q[6] < 4)
        q[6]++;
      else if (ioncharge == 0) {
        if (q[9] < 2)
          q[9]++;
        else if (q[7] < 4)
          q[7]++;
        else if (q[8] < 6)
          q[8]++;
        else {
          *fail = 1;
          return 0.;
        }
      } else if (ioncharge == 1) {
        if (q[9] < 1)
          q[9]++;
        else if (q[7] < 4)
          q[7]++;
        else if (q[8] < 6)
          q[8]++;
        else {
          *fail = 1;
          return 0.;
        }
      } else if (ioncharge > 1) {
        if (q[7] < 4)
          q[7]++;
        else if (q[8] < 6)
          q[8]++;
        else {
          *fail = 1;
          return 0.;
        }
      }
    }
    total = 0.0;
    for (int electron_loop = 0; electron_loop < kMNtShells; electron_loop++) {
      const double electronsinshell = q[electron_loop];
      if (electronsinshell > 0) {
        double use2 = nt->electron_binding[(Zel - 1) * kMNtShells + electron_loop];
        const double use3 = c.at->ion_ionpot[uion(c, e, i)];
        if (use2 <= 0) {
          use2 = nt->electron_binding[(Zel - 1) * kMNtShells + electron_loop - 1];
          if (electron_loop != 8) {
            *fail = 1;
            return 0.;
          }
        }
        if (use2 < use3)
          total += electronsinshell / use3;
        else
          total += electronsinshell / use2;
      }
    }
  } else {
    total = 0.0;
  }
  return total;
}
// nonthermal.cc:1311-1331 get_oneoverw
double sf_oneoverw(const Ctx &c, const NlteRun &r, int e, int i, int mgi, int *fail) {
  double Zbar = 0.0;
  for (int ie = 0; ie < c.at->nelements; ie++)
    Zbar += r.in->elem_abundance[(size_t)mgi * c.at->nelements + ie] * c.at->elem_anumber[ie];
  const double Aconst = 1.33e-14 * ARTIS_EV * ARTIS_EV;
  const double binding = sf_mean_binding_energy(c, r.nt, e, i, fail);
  return Aconst * binding / Zbar / (2 * 3.14159 * pow(ARTIS_QE, 4));
}

// the non-thermal solution of one cell: nt_solution[mgi] (nonthermal.cc:123-146)
struct NtSol {
  float *frac_heating, *frac_ionization, *frac_excitation, *nneperion_when_solved, *eff_ionpot;
  int32_t *timestep_last_solved;
  double *fracdep_ionization_ion;
  float *prob, *ionen;
};
NtSol nt_sol(const Ctx &c, const NlteRun &r, int mgi) {
  const size_t ni = c.at->nions_total;
  NtSol s;
  s.frac_heating = r.in->nt_frac_heating + mgi;
  s.frac_ionization = r.in->nt_frac_ionization + mgi;
  s.frac_excitation = r.in->nt_frac_excitation + mgi;
  s.nneperion_when_solved = r.in->nt_nneperion_when_solved + mgi;
  s.timestep_last_solved = r.in->nt_timestep_last_solved + mgi;
  s.eff_ionpot = r.in->nt_eff_ionpot + (size_t)mgi * ni;
  s.fracdep_ionization_ion = r.in->nt_fracdep_ionization_ion + (size_t)mgi * ni;
  s.prob = r.g->nt_prob.data() + (size_t)mgi * ni * (kNtMaxAuger + 1);
  s.ionen = r.g->nt_ionen.data() + (size_t)mgi * ni * (kNtMaxAuger + 1);
  return s;
}
// nonthermal.cc:439-460 zero_all_effionpot
void sf_zero_all_effionpot(const Ctx &c, const NtSol &s) {
  for (int u = 0; u < c.at->nions_total; u++) {
    s.eff_ionpot[u] = 0.;
    s.prob[u * (kNtMaxAuger + 1)] = 1.;
    s.ionen[u * (kNtMaxAuger + 1)] = 1.;
    for (int a = 1; a <= kNtMaxAuger; a++) {
      s.prob[u * (kNtMaxAuger + 1) + a] = 0.;
      s.ionen[u * (kNtMaxAuger + 1) + a] = 0.;
    }
  }
}

// Upper-triangular system U y = b (U row-major [n * n]): GSL LU_solve with the identity permutation (the strictly
// lower part of U is zero, so the unit-lower solve is the identity) and a column-oriented back substitution (D11)
void sf_backsub(const double *U, int n, double *x) {
  for (int j = n - 1; j >= 0; j--) {
    x[j] = x[j] / U[(size_t)j * n + j];
    for (int i = 0; i < j; i++) x[i] -= U[(size_t)i * n + j] * x[j];
  }
}
// nonthermal.cc:2461-2520 sfmatrix_solve: 10 passes, every pass after the first one gsl_linalg_LU_refine, the
// solution with the smallest max-norm residual kept
void sf_solve(const double *U, const double *b, int n, double *y) {
  std::vector<double> x(b, b + n), best(n), work(n), res(n);
  sf_backsub(U, n, x.data());
  double error_best = -1.;
  for (int iteration = 0; iteration < 10; iteration++) {
    if (iteration > 0) {
      // gsl_linalg_LU_refine: work = A x - b (dgemv, beta = -1), LU_svx(work), x -= work (daxpy)
      for (int i = 0; i < n; i++) {
        double temp = 0.;
        for (int j = i; j < n; j++) temp += x[j] * U[(size_t)i * n + j];
        work[i] = -b[i] + temp;
      }
      sf_backsub(U, n, work.data());
      for (int i = 0; i < n; i++) x[i] += -1.0 * work[i];
    }
    for (int i = 0; i < n; i++) {
      double temp = 0.;
      for (int j = i; j < n; j++) temp += x[j] * U[(size_t)i * n + j];
      res[i] = -b[i] + temp;
    }
    int imax = 0;  // gsl_blas_idamax: the first index of the largest |r_i|
    double amax = -1.;
    for (int i = 0; i < n; i++)
      if (fabs(res[i]) > amax) {
        amax = fabs(res[i]);
        imax = i;
      }
    const double error = fabs(res[imax]);
    if (error < error_best || error_best < 0.) {
      best = x;
      error_best = error;
    }
  }
  for (int i = 0; i < n; i++) y[i] = best[i];
}

// nonthermal.cc:1333-1360 calculate_nt_frac_ionization_shell
double sf_frac_ionization_shell(const Ctx &c, const NlteRun &r, int mgi, int e, int i, int k, const double *y) {
  const double nnion = ionstagepop(c, mgi, e, i);
  const double ionpot_ev = r.nt->ionpot_ev[k];
  std::vector<double> xs(r.sf.n);
  sf_xs_ionization_vector(r.sf, r.nt, k, xs.data());
  double y_dot = 0.;
  for (int j = 0; j < r.sf.n; j++) y_dot += y[j] * xs[j];
  y_dot *= r.sf.delta_e;
  return nnion * ionpot_ev * y_dot / r.sf.E_init_ev;
}
// nonthermal.cc:1430-1556 calculate_eff_ionpot_auger_rates
void sf_eff_ionpot_auger_rates(const Ctx &c, const NlteRun &r, int mgi, int e, int i, const double *y, const NtSol &s,
                               int *fail) {
  const int Z = c.at->elem_anumber[e];
  const int ionstage = get_ionstage(c, e, i);
  const int u = uion(c, e, i);
  const double nnion = ionstagepop(c, mgi, e, i);
  const double tot_nion = nl_get_nntot(c, r, mgi);
  const double X_ion = nnion / tot_nion;
  double eta_nauger_ionize_over_ionpot_sum[kNtMaxAuger + 1], eta_nauger_ionize_sum[kNtMaxAuger + 1];
  for (int a = 0; a <= kNtMaxAuger; a++) {
    eta_nauger_ionize_over_ionpot_sum[a] = 0.;
    s.prob[u * (kNtMaxAuger + 1) + a] = 0.;
    eta_nauger_ionize_sum[a] = 0.;
    s.ionen[u * (kNtMaxAuger + 1) + a] = 0.;
  }
  double eta_over_ionpot_sum = 0., eta_sum = 0.;
  int matching = 0;
  for (int k = 0; k < r.nt->nshells; k++) {
    if (!shell_matches(r.nt, k, Z, ionstage)) continue;
    matching++;
    const double frac_ionization_shell = sf_frac_ionization_shell(c, r, mgi, e, i, k, y);
    eta_sum += frac_ionization_shell;
    const double ionpot_shell = r.nt->ionpot_ev[k] * ARTIS_EV;
    const double eta_over_ionpot = frac_ionization_shell / ionpot_shell;  // NT_USE_VALENCE_IONPOTENTIAL false
    eta_over_ionpot_sum += eta_over_ionpot;
    for (int a = 0; a <= kNtMaxAuger; a++) {
      eta_nauger_ionize_over_ionpot_sum[a] += eta_over_ionpot * r.nt->prob_num_auger[k * (kNtMaxAuger + 1) + a];
      eta_nauger_ionize_sum[a] += frac_ionization_shell * r.nt->prob_num_auger[k * (kNtMaxAuger + 1) + a];
    }
  }
  if (kNtMaxAuger > 0 && matching > 0) {
    const int nions = get_nions(c, e);
    if (i < nions - 1) {
      for (int a = 0; a <= kNtMaxAuger; a++) {
        if (i + 1 + a < nions) {
          s.prob[u * (kNtMaxAuger + 1) + a] = eta_nauger_ionize_over_ionpot_sum[a] / eta_over_ionpot_sum;
          s.ionen[u * (kNtMaxAuger + 1) + a] = eta_nauger_ionize_sum[a] / eta_sum;
        } else {
          s.prob[u * (kNtMaxAuger + 1) + nions - 1 - i - 1] += eta_nauger_ionize_over_ionpot_sum[a] / eta_over_ionpot_sum;
          s.ionen[u * (kNtMaxAuger + 1) + nions - 1 - i - 1] += eta_nauger_ionize_sum[a] / eta_sum;
          s.prob[u * (kNtMaxAuger + 1) + a] = 0;
          s.ionen[u * (kNtMaxAuger + 1) + a] = 0.;
        }
      }
    }
  } else {
    s.prob[u * (kNtMaxAuger + 1)] = 1.;
    s.ionen[u * (kNtMaxAuger + 1)] = 1.;
  }
  if (matching > 0) {
    double eff_ionpot = X_ion / eta_over_ionpot_sum;
    if (!std::isfinite(eff_ionpot)) eff_ionpot = 0.;
    s.eff_ionpot[u] = eff_ionpot;
  } else {
    s.eff_ionpot[u] = 1. / sf_oneoverw(c, r, e, i, mgi, fail);
  }
}
// nonthermal.cc:1714-1744 calculate_nt_excitation_ratecoeff_perdeposition
double sf_excitation_ratecoeff_perdeposition(const Ctx &c, const NlteRun &r, const double *y, int li,
                                             double statweight_lower, double epsilon_trans) {
  std::vector<double> xs(r.sf.n);
  if (sf_xs_excitation_vector(c, r.sf, xs.data(), li, statweight_lower, epsilon_trans) >= 0) {
    double y_dot = 0.;
    for (int j = 0; j < r.sf.n; j++) y_dot += xs[j] * y[j];
    y_dot *= r.sf.delta_e;
    return y_dot / r.sf.E_init_ev / ARTIS_EV;
  }
  return 0.;
}
// nonthermal.cc:1996-2280 analyse_sf_solution (NT_EXCITATION_ON false; D12)
void sf_analyse(const Ctx &c, const NlteRun &r, int mgi, const double *y, const NtSol &s, int *fail) {
  double frac_excitation_total = 0., frac_ionization_total = 0.;
  for (int e = 0; e < c.at->nelements; e++) {
    const int Z = c.at->elem_anumber[e];
    const int nions = get_nions(c, e);
    for (int i = 0; i < nions; i++) {
      const int u = uion(c, e, i);
      const int ionstage = get_ionstage(c, e, i);
      const double nnion = ionstagepop(c, mgi, e, i);
      if (nnion <= 0.) continue;
      double frac_ionization_ion = 0., frac_excitation_ion = 0.;
      sf_eff_ionpot_auger_rates(c, r, mgi, e, i, y, s, fail);
      for (int k = 0; k < r.nt->nshells; k++)
        if (shell_matches(r.nt, k, Z, ionstage)) frac_ionization_ion += sf_frac_ionization_shell(c, r, mgi, e, i, k, y);
      if (i < nions - 1) {
        s.fracdep_ionization_ion[u] = frac_ionization_ion;
        frac_ionization_total += frac_ionization_ion;
      } else {
        s.fracdep_ionization_ion[u] = 0.;
      }
      const int nlevels_all = get_nlevels(c, e, i);
      const int nlevels = (nlevels_all > kNtExcMaxLower) ? kNtExcMaxLower : nlevels_all;
      for (int lower = 0; lower < nlevels; lower++) {
        const double statweight_lower = stat_weight(c, e, i, lower);
        const int ul = ulev(c, e, i, lower);
        const int nuptrans = c.at->level_nuptrans[ul];
        const double nnlevel = calculate_levelpop(c, mgi, e, i, lower);
        const double epsilon_lower = epsilon(c, e, i, lower);
        for (int t = 0; t < nuptrans; t++) {
          const int li = c.at->uptrans_lineindex[c.at->level_uptrans_offset[ul] + t];
          const int upper = c.at->line_upperlevelindex[li];
          if (upper >= kNtExcMaxUpper) continue;
          const double epsilon_trans = epsilon(c, e, i, upper) - epsilon_lower;
          const double nt_frac_excitation_perlevelpop =
              epsilon_trans * sf_excitation_ratecoeff_perdeposition(c, r, y, li, statweight_lower, epsilon_trans);
          frac_excitation_ion += nnlevel * nt_frac_excitation_perlevelpop;
        }
      }
      if (frac_excitation_ion > 1. || !std::isfinite(frac_excitation_ion)) frac_excitation_ion = 0.;
      frac_excitation_total += frac_excitation_ion;
    }
  }
  *s.frac_excitation = frac_excitation_total;
  *s.frac_ionization = frac_ionization_total;
  *s.frac_heating = 1. - frac_excitation_total - frac_ionization_total;
}

// the Spencer-Fano matrix (row-major, upper triangular) and right-hand side of solve_spencerfano
// (nonthermal.cc:2617-2674), with sfmatrix_add_excitation (2282-2341) and sfmatrix_add_ionization (2343-2459)
void sf_build(const Ctx &c, const NlteRun &r, int mgi, std::vector<double> &M, std::vector<double> &rhs) {
  const SfGrid &s = r.sf;
  const int n = s.n;
  const double DE = s.delta_e;
  M.assign((size_t)n * n, 0.);
  rhs.assign(n, 0.);
  const float nne = r.g->nne[mgi];
  for (int i = 0; i < n; i++) {
    const double en = s.envec[i];
    M[(size_t)i * n + i] += sf_electron_loss_rate(en * ARTIS_EV, nne) / ARTIS_EV;
    double source_integral_to_SF_EMAX = 0.;
    if (i < n - 1) {
      double dasum = 0.;
      for (int j = i + 1; j < n; j++) dasum += fabs(s.sourcevec[j]);
      source_integral_to_SF_EMAX = dasum * DE;
    }
    rhs[i] = source_integral_to_SF_EMAX;
  }
  const double tot_nion = nl_get_nntot(c, r, mgi);
  std::vector<double> xs(n), int_eps_upper(n), prefactors(n);
  for (int e = 0; e < c.at->nelements; e++) {
    const int Z = c.at->elem_anumber[e];
    const int nions = get_nions(c, e);
    for (int i = 0; i < nions; i++) {
      const double nnion = ionstagepop(c, mgi, e, i);
      if (nnion < kMinIonFraction * tot_nion) continue;
      const int ionstage = get_ionstage(c, e, i);
      // excitation
      {
        const int nlevels_all = get_nlevels(c, e, i);
        const int nlevels = (nlevels_all > kNtExcMaxLower) ? kNtExcMaxLower : nlevels_all;
        for (int lower = 0; lower < nlevels; lower++) {
          const double statweight_lower = stat_weight(c, e, i, lower);
          const double nnlevel = calculate_levelpop(c, mgi, e, i, lower);
          const double epsilon_lower = epsilon(c, e, i, lower);
          const int ul = ulev(c, e, i, lower);
          for (int t = 0; t < c.at->level_nuptrans[ul]; t++) {
            const int li = c.at->uptrans_lineindex[c.at->level_uptrans_offset[ul] + t];
            const int upper = c.at->line_upperlevelindex[li];
            if (upper >= kNtExcMaxUpper) continue;
            const double epsilon_trans = epsilon(c, e, i, upper) - epsilon_lower;
            const double epsilon_trans_ev = epsilon_trans / ARTIS_EV;
            if (epsilon_trans_ev < s.emin) continue;
            const int xsstartindex = sf_xs_excitation_vector(c, s, xs.data(), li, statweight_lower, epsilon_trans);
            if (xsstartindex < 0) continue;
            for (int j = 0; j < n; j++) xs[j] *= DE;  // gsl_blas_dscal(DELTA_E)
            for (int ii = 0; ii < n; ii++) {
              const double en = s.envec[ii];
              const int stopindex = sf_lteq(s, en + epsilon_trans_ev);
              const int startindex = ii > xsstartindex ? ii : xsstartindex;
              for (int j = startindex; j < stopindex; j++) M[(size_t)ii * n + j] += nnlevel * xs[j];
              const double delta_en_actual = (en + epsilon_trans_ev - s.envec[stopindex]);
              M[(size_t)ii * n + stopindex] += nnlevel * xs[stopindex] * delta_en_actual / DE;
            }
          }
        }
      }
      // ionisation
      if (i < nions - 1) {
        for (int k = 0; k < r.nt->nshells; k++) {
          if (!shell_matches(r.nt, k, Z, ionstage)) continue;
          const double ionpot_ev = r.nt->ionpot_ev[k];
          const double en_auger_ev = r.nt->en_auger_ev[k];
          const double J = sf_get_J(Z, ionstage, ionpot_ev);
          const int xsstartindex = sf_xs_ionization_vector(s, r.nt, k, xs.data());
          for (int j = xsstartindex; j < n; j++) {
            const double endash = s.envec[j];
            const double epsilon_upper = std::min((endash + ionpot_ev) / 2, endash);
            int_eps_upper[j] = atan((epsilon_upper - ionpot_ev) / J);
            prefactors[j] = xs[j] * nnion / atan((endash - ionpot_ev) / 2 / J);
          }
          for (int ii = 0; ii < n; ii++) {
            const double en = s.envec[ii];
            const int jstart = ii > xsstartindex ? ii : xsstartindex;
            for (int j = jstart; j < n; j++) {
              const double endash = s.envec[j];
              const double epsilon_lower = std::max(endash - en, ionpot_ev);
              const double int_eps_lower = atan((epsilon_lower - ionpot_ev) / J);
              if (int_eps_lower <= int_eps_upper[j])
                M[(size_t)ii * n + j] += prefactors[j] * (int_eps_upper[j] - int_eps_lower) * DE;
            }
            const double int_eps_lower2 = atan(en / J);
            if (2 * en + ionpot_ev <= s.emax) {
              const int secondintegralstartindex = sf_lteq(s, 2 * en + ionpot_ev);
              // D10: terms below xsstartindex are skipped (their prefactor is uninitialised in the reference)
              for (int j = std::max(secondintegralstartindex, xsstartindex); j < n; j++) {
                if (int_eps_lower2 <= int_eps_upper[j])
                  M[(size_t)ii * n + j] -= prefactors[j] * (int_eps_upper[j] - int_eps_lower2) * DE;
              }
            }
          }
          // SF_AUGER_CONTRIBUTION_ON, SF_AUGER_CONTRIBUTION_DISTRIBUTE_EN false
          const int augerstopindex = sf_gteq(s, en_auger_ev);
          for (int ii = 0; ii < augerstopindex; ii++) {
            const int jstart = ii > xsstartindex ? ii : xsstartindex;
            for (int j = jstart; j < n; j++) M[(size_t)ii * n + j] -= nnion * xs[j];
          }
        }
      }
    }
  }
}

// nonthermal.cc:2522-2713 solve_spencerfano
void nl_solve_spencerfano(const Ctx &c, const NlteRun &r, int mgi, int timestep, int *fail, std::vector<double> *y_out) {
  const NtSol s = nt_sol(c, r, mgi);
  bool skip_solution = false;
  if (timestep < r.p->num_lte_timesteps + 1)
    skip_solution = true;
  else if (r.in->deposition_rate_density[mgi] / ARTIS_EV < 0.)  // MINDEPRATE 0
    skip_solution = true;
  if (skip_solution) {
    *s.frac_heating = 0.97;
    *s.frac_ionization = 0.03;
    *s.frac_excitation = 0.;
    *s.nneperion_when_solved = -1.;
    *s.timestep_last_solved = -1;
    sf_zero_all_effionpot(c, s);
    return;
  }
  const float nne = r.g->nne[mgi];
  const double nne_per_ion = nne / nl_get_nntot(c, r, mgi);
  const double nne_per_ion_last = *s.nneperion_when_solved;
  const double nne_per_ion_fracdiff = fabs((nne_per_ion_last / nne_per_ion) - 1.);
  const int timestep_last_solved = *s.timestep_last_solved;
  if ((nne_per_ion_fracdiff < 0.05) && (timestep - timestep_last_solved <= 0) &&
      timestep_last_solved > r.p->num_lte_timesteps)
    return;
  *s.nneperion_when_solved = nne_per_ion;
  *s.timestep_last_solved = timestep;
  std::vector<double> M, rhs, y(r.sf.n);
  sf_build(c, r, mgi, M, rhs);
  sf_solve(M.data(), rhs.data(), r.sf.n, y.data());
  sf_analyse(c, r, mgi, y.data(), s, fail);
  if (y_out) *y_out = y;
}

// nonthermal.cc:1567-1582, 1684-1712 nt_ionization_ratecoeff (NT_SOLVE_SPENCERFANO)
double nl_nt_ionization_ratecoeff(const Ctx &c, const NlteRun &r, int mgi, int e, int i, int *fail) {
  const double deposition_rate_density = r.in->deposition_rate_density[mgi];
  double Y_nt = 0.;
  if (deposition_rate_density > 0.)
    Y_nt = deposition_rate_density / nl_get_nntot(c, r, mgi) / r.in->nt_eff_ionpot[nix(c, mgi, e, i)];
  if (!std::isfinite(Y_nt) || Y_nt <= 0)
    return deposition_rate_density / nl_get_nntot(c, r, mgi) * sf_oneoverw(c, r, e, i, mgi, fail);
  return Y_nt;
}
// the Y_nt of every ion into the state the NLTE matrix and phi read (c.cs->nt_ionization_ratecoeff)
void nl_store_nt_rates(const Ctx &c, const NlteRun &r, int mgi, int *fail) {
  for (int e = 0; e < c.at->nelements; e++)
    for (int i = 0; i < get_nions(c, e); i++)
      r.g->ntY[nix(c, mgi, e, i)] = (i < get_nions(c, e) - 1) ? nl_nt_ionization_ratecoeff(c, r, mgi, e, i, fail) : 0.;
}

// --------------------------------------------------------------------------------------------- T_e solver
// thermalbalance.cc:218-346 (DIRECT_COL_HEAT)
void nl_calculate_heating_rates(const Ctx &c, const NlteRun &r, int mgi, const std::vector<double> &coeff, TeRates *hc) {
  double C_deexc = 0., bfheating = 0.;
  const float T_e = r.g->Te[mgi];
  const float nne = r.g->nne[mgi];
  for (int e = 0; e < c.at->nelements; e++) {
    const int nions = get_nions(c, e);
    for (int i = 0; i < nions; i++) C_deexc += te_heating_ion_coll_deexc(c, mgi, e, i, T_e, nne);
    for (int i = 0; i < nions - 1; i++)
      for (int level = 0; level < get_ionisinglevels(c, e, i); level++)
        bfheating += calculate_levelpop(c, mgi, e, i, level) * coeff[ulev(c, e, i, level)];
  }
  hc->heating_collisional = C_deexc;
  hc->heating_bf = bfheating;
  // heating_ff: the normalised ffheatingestimator, set by nl_te_eqn
}
// thermalbalance.cc:348-395 with NLTE_POPS_ALL_IONS_SIMULTANEOUS: calculate_electron_densities
double nl_te_eqn(const Ctx &c, const NlteRun &r, int mgi, double T_e, const std::vector<double> &coeff, double ffheat,
                 TeRates *hc) {
  r.g->Te[mgi] = T_e;
  const double nntot = nl_calculate_electron_densities(c, r, mgi);
  te_calculate_cooling_rates(c, mgi, hc, nullptr, nullptr);
  nl_calculate_heating_rates(c, r, mgi, coeff, hc);
  hc->heating_ff = ffheat;
  if (r.p->do_rlc_est == 3) {
    hc->heating_dep = r.in->deposition_rate_density[mgi] * (double)r.in->nt_frac_heating[mgi];
  } else {
    hc->heating_dep = 0.;
  }
  const double p = nntot * ARTIS_KB * T_e;
  const double volumetmin = r.in->vol_init[mgi];
  const double dV = 3 * volumetmin / pow(r.p->tmin, 3) * pow(r.p->t_current_te, 2);
  const double V = volumetmin * pow(r.p->t_current_te / r.p->tmin, 3);
  hc->cooling_adiabatic = p * dV / V;
  const double total_heating_rate = hc->heating_ff + hc->heating_bf + hc->heating_collisional + hc->heating_dep;
  const double total_coolingrate = hc->cooling_ff + hc->cooling_fb + hc->cooling_collisional + hc->cooling_adiabatic;
  return total_heating_rate - total_coolingrate;
}
// thermalbalance.cc:397-597; -2 on GSL's abort paths
int nl_call_T_e_finder(const Ctx &c, const NlteRun &r, int mgi, const std::vector<double> &coeff, double ffheat,
                       TeRates *hc) {
  const double T_min = r.p->T_min, T_max = r.p->T_max;
  const double T_e_old = r.g->Te[mgi];
  auto f = [&](double T) { return nl_te_eqn(c, r, mgi, T, coeff, ffheat, hc); };
  double thermalmin = f(T_min);
  double thermalmax = f(T_max);
  if (!std::isfinite(thermalmin) || !std::isfinite(thermalmax)) thermalmax = thermalmin = -1;
  double T_e = 0.;
  if (thermalmin * thermalmax < 0) {
    GslBrent s;
    if (gsl_brent_set(s, f, T_min, T_max) != 0) return -2;
    for (int iternum = 0; iternum < 100; iternum++) {
      if (gsl_brent_iterate(s, f) != 0) return -2;
      T_e = s.root;
      if (gsl_test_interval(s.x_lower, s.x_upper, 0, r.p->accuracy) != 1) break;
    }
  } else if (thermalmax < 0) {
    T_e = T_min;
  } else {
    T_e = T_max;
  }
  if (T_e > 2 * T_e_old) {
    T_e = 2 * T_e_old;
    if (T_e > T_max) T_e = T_max;
  } else if (T_e < 0.5 * T_e_old) {
    T_e = 0.5 * T_e_old;
    if (T_e < T_min) T_e = T_min;
  }
  r.g->Te[mgi] = T_e;
  f(T_e);
  return 0;
}

// ------------------------------------------------------------------------------------------ NLTE populations
// nltepop.cc:24-38 get_nlte_vector_index
inline int nlte_vector_index(const Ctx &c, int e, int i, int l) {
  const int gs_index = c.at->ion_first_nlte[uion(c, e, i)] - c.at->ion_first_nlte[uion(c, e, 0)] + i;
  const int nn = get_nlevels_nlte(c, e, i);
  return gs_index + ((l <= nn) ? l : (nn + 1));
}
inline bool ion_has_superlevel(const Ctx &c, int e, int i) { return get_nlevels(c, e, i) > get_nlevels_nlte(c, e, i) + 1; }
// nltepop.cc:40-51 (the first level mapping to index)
void nlte_ion_level_of_index(const Ctx &c, int index, int e, int *ion, int *level) {
  for (int dion = 0; dion < get_nions(c, e); dion++)
    for (int dlevel = 0; dlevel < get_nlevels(c, e, dion); dlevel++)
      if (nlte_vector_index(c, e, dion, dlevel) == index) {
        *ion = dion;
        *level = dlevel;
        return;
      }
}
// nltepop.cc:376-389
void nlte_reset_element(const Ctx &c, const NlteRun &r, int mgi, int e) {
  double *row = r.g->nlte_pops.data() + (size_t)mgi * c.at->total_nlte_levels;
  for (int i = 0; i < get_nions(c, e); i++) {
    const int nlte_start = c.at->ion_first_nlte[uion(c, e, i)];
    const int nn = get_nlevels_nlte(c, e, i);
    for (int level = 1; level < nn; level++) row[nlte_start + level - 1] = -1.0;
    if (ion_has_superlevel(c, e, i)) row[nlte_start + nn] = -1.0;
  }
}

// LU decomposition with partial pivoting, right-looking (GSL <= 2.6 linalg/lu.c; D11); A column-major [n * n]
void nlte_lu_decomp(double *A, int n, std::vector<int> &perm) {
  auto a = [&](int r_, int c_) -> double & { return A[(size_t)c_ * n + r_]; };
  perm.resize(n);
  for (int j = 0; j < n; j++) perm[j] = j;
  for (int j = 0; j < n - 1; j++) {
    double max = fabs(a(j, j));
    int i_pivot = j;
    for (int i = j + 1; i < n; i++) {
      const double aij = fabs(a(i, j));
      if (aij > max) {
        max = aij;
        i_pivot = i;
      }
    }
    if (i_pivot != j) {
      for (int k = 0; k < n; k++) std::swap(a(j, k), a(i_pivot, k));
      std::swap(perm[j], perm[i_pivot]);
    }
    const double ajj = a(j, j);
    if (ajj != 0.0) {
      for (int i = j + 1; i < n; i++) {
        const double aij = a(i, j) / ajj;
        a(i, j) = aij;
        for (int k = j + 1; k < n; k++) a(i, k) = a(i, k) - aij * a(j, k);
      }
    }
  }
}
// gsl_linalg_LU_svx: x := P b, then L (unit, dtrsv order) and U (column-oriented, D11)
void nlte_lu_svx(const double *LU, int n, const std::vector<int> &perm, double *x) {
  std::vector<double> t(x, x + n);
  for (int i = 0; i < n; i++) x[i] = t[perm[i]];  // gsl_permute_vector: x'_i = x_{p_i}
  for (int i = 0; i < n; i++) {
    double tmp = x[i];
    for (int j = 0; j < i; j++) tmp -= LU[(size_t)j * n + i] * x[j];
    x[i] = tmp;
  }
  for (int j = n - 1; j >= 0; j--) {
    x[j] = x[j] / LU[(size_t)j * n + j];
    for (int i = 0; i < j; i++) x[i] -= LU[(size_t)j * n + i] * x[j];
  }
}
// residual A x - b (gsl_blas_dgemv NoTrans, alpha 1, beta -1; row-serial sums), A column-major
void nlte_residual(const double *A, int n, const double *x, const double *b, double *res) {
  for (int i = 0; i < n; i++) {
    double temp = 0.;
    for (int j = 0; j < n; j++) temp += x[j] * A[(size_t)j * n + i];
    res[i] = -b[i] + temp;
  }
}
// nltepop.cc:656-677, 679-796 nltepop_matrix_solve; false: singular
bool nlte_matrix_solve(const double *A, const double *b, int n, double *popvec, const double *norm) {
  std::vector<double> LU(A, A + (size_t)n * n);
  std::vector<int> perm;
  nlte_lu_decomp(LU.data(), n, perm);
  for (int i = 0; i < n; i++)
    if (LU[(size_t)i * n + i] == 0) return false;
  std::vector<double> x(b, b + n), best(n), work(n), res(n);
  nlte_lu_svx(LU.data(), n, perm, x.data());
  double error_best = -1.;
  for (int iteration = 0; iteration < 10; iteration++) {
    if (iteration > 0) {
      nlte_residual(A, n, x.data(), b, work.data());
      nlte_lu_svx(LU.data(), n, perm, work.data());
      for (int i = 0; i < n; i++) x[i] += -1.0 * work[i];
    }
    nlte_residual(A, n, x.data(), b, res.data());
    int imax = 0;
    double amax = -1.;
    for (int i = 0; i < n; i++)
      if (fabs(res[i]) > amax) {
        amax = fabs(res[i]);
        imax = i;
      }
    const double error = fabs(res[imax]);
    if (error < error_best || error_best < 0.) {
      best = x;
      error_best = error;
    }
    if (error < 1e-40) break;
  }
  for (int i = 0; i < n; i++) {
    popvec[i] = best[i] * norm[i];
    if (popvec[i] < 0.0) popvec[i] = norm[i];
  }
  return true;
}

thread_local std::vector<double> tl_raw_matrix;  // the last rate matrix before normalisation (ORACLE_NL_DUMP)

// the element's rate matrix, normalised, column-major, with its balance vector and LTE normalisation
// (nltepop.cc:391-628, 832-920): the five process matrices summed in the reference's order (NT excitation is zero,
// NT_EXCITATION_ON false)
int nlte_build(const Ctx &c, const NlteRun &r, int mgi, int e, std::vector<double> &A, std::vector<double> &b,
               std::vector<double> &norm, std::vector<double> &slpf) {
  const int nions = get_nions(c, e);
  int D = 0;
  slpf.assign(nions, 0.);
  for (int i = 0; i < nions; i++) {
    const int nn = get_nlevels_nlte(c, e, i);
    if (ion_has_superlevel(c, e, i)) {
      D += nn + 2;
      for (int level = nn + 1; level < get_nlevels(c, e, i); level++) slpf[i] += superlevel_boltzmann(c, mgi, e, i, level);
    } else {
      D += nn + 1;
    }
  }
  std::vector<double> rad_bb((size_t)D * D, 0.), coll_bb((size_t)D * D, 0.), rad_bf((size_t)D * D, 0.),
      coll_bf((size_t)D * D, 0.), ntcoll_bf((size_t)D * D, 0.);
  auto at = [&](std::vector<double> &m, int row, int col) -> double & { return m[(size_t)col * D + row]; };
  const float T_e = r.g->Te[mgi];
  const float nne = r.g->nne[mgi];
  const double t_mid = r.p->t_mid;
  ThreadCache tc;  // the level populations of the current state (use_cellhist false in update_grid)
  tc.pops.resize(c.at->nlevels_total);
  int64_t ntg = 0;  // photoionisation target slots (level_phixstargets_offset + t)
  for (int lv = 0; lv < c.at->nlevels_total; lv++) ntg += c.at->level_nphixstargets[lv];
  tc.corrphotoioncoeff.assign(ntg + 1, -99.);
  for (int ie = 0; ie < c.at->nelements; ie++)
    for (int ii = 0; ii < get_nions(c, ie); ii++)
      for (int l = 0; l < get_nlevels(c, ie, ii); l++) tc.pops[ulev(c, ie, ii, l)] = calculate_levelpop(c, mgi, ie, ii, l);
  tc.cellnumber = mgi;
  for (int i = 0; i < nions; i++) {
    const int nlevels = get_nlevels(c, e, i);
    const int nn = get_nlevels_nlte(c, e, i);
    std::vector<double> s_renorm(nlevels, 0.);
    for (int level = 0; level <= nn && level < nlevels; level++) s_renorm[level] = 1.0;
    for (int level = nn + 1; level < nlevels; level++) s_renorm[level] = superlevel_boltzmann(c, mgi, e, i, level) / slpf[i];
    // nltepop.cc:421-505 nltepop_matrix_add_boundbound
    for (int level = 0; level < nlevels; level++) {
      const int level_index = nlte_vector_index(c, e, i, level);
      const double epsilon_level = epsilon(c, e, i, level);
      const double statweight = stat_weight(c, e, i, level);
      const int ul = ulev(c, e, i, level);
      for (int k = 0; k < c.at->level_ndowntrans[ul]; k++) {
        const int li = c.at->downtrans_lineindex[c.at->level_downtrans_offset[ul] + k];
        const int lower = c.at->line_lowerlevelindex[li];
        const double epsilon_trans = epsilon_level - epsilon(c, e, i, lower);
        const double R = rad_deexcitation_ratecoeff(c, tc, e, i, level, lower, epsilon_trans, li, t_mid) * s_renorm[level];
        const double C = col_deexcitation_ratecoeff(c, T_e, nne, epsilon_trans, li, stat_weight(c, e, i, lower), statweight) *
                         s_renorm[level];
        const int upper_index = level_index, lower_index = nlte_vector_index(c, e, i, lower);
        at(rad_bb, upper_index, upper_index) -= R;
        at(rad_bb, lower_index, upper_index) += R;
        at(coll_bb, upper_index, upper_index) -= C;
        at(coll_bb, lower_index, upper_index) += C;
      }
      for (int k = 0; k < c.at->level_nuptrans[ul]; k++) {
        const int li = c.at->uptrans_lineindex[c.at->level_uptrans_offset[ul] + k];
        const int upper = c.at->line_upperlevelindex[li];
        const double epsilon_trans = epsilon(c, e, i, upper) - epsilon_level;
        const double R = rad_excitation_ratecoeff(c, tc, mgi, e, i, level, upper, epsilon_trans, li, t_mid) * s_renorm[level];
        const double C = col_excitation_ratecoeff(c, T_e, nne, li, epsilon_trans, statweight, stat_weight(c, e, i, upper)) *
                         s_renorm[level];
        const int lower_index = level_index, upper_index = nlte_vector_index(c, e, i, upper);
        at(rad_bb, lower_index, lower_index) -= R;
        at(rad_bb, upper_index, lower_index) += R;
        at(coll_bb, lower_index, lower_index) -= C;
        at(coll_bb, upper_index, lower_index) += C;
      }
    }
    if (i < nions - 1) {
      // nltepop.cc:507-562 nltepop_matrix_add_ionisation
      const int maxrecombininglevel = get_maxrecombininglevel(c, e, i + 1);
      for (int level = 0; level < get_ionisinglevels(c, e, i); level++) {
        const int lower_index = nlte_vector_index(c, e, i, level);
        const double epsilon_current = epsilon(c, e, i, level);
        for (int t = 0; t < get_nphixstargets(c, e, i, level); t++) {
          const int upper = get_phixsupperlevel(c, e, i, level, t);
          const int upper_index = nlte_vector_index(c, e, i + 1, upper);
          const double epsilon_trans = epsilon(c, e, i + 1, upper) - epsilon_current;
          const double R_ionisation = get_corrphotoioncoeff(c, tc, e, i, level, t, mgi);
          const double C_ionisation = col_ionization_ratecoeff(c, T_e, nne, e, i, level, t, epsilon_trans);
          at(rad_bf, lower_index, lower_index) -= R_ionisation * s_renorm[level];
          at(rad_bf, upper_index, lower_index) += R_ionisation * s_renorm[level];
          at(coll_bf, lower_index, lower_index) -= C_ionisation * s_renorm[level];
          at(coll_bf, upper_index, lower_index) += C_ionisation * s_renorm[level];
          if (upper <= maxrecombininglevel) {
            const double R_recomb = rad_recombination_ratecoeff(c, T_e, nne, e, i + 1, upper, level);
            const double C_recomb = col_recombination_ratecoeff(c, mgi, e, i + 1, upper, level, epsilon_trans);
            // nltepop.cc:551-554 index s_renorm -- the array of the lower ion being processed -- with the upper ion's
            // level number; restated as is.  D13: an index past that array (a read beyond the reference's
            // allocation) counts as 0.
            const double sr = (upper < nlevels) ? s_renorm[upper] : 0.;
            at(rad_bf, upper_index, upper_index) -= R_recomb * sr;
            at(rad_bf, lower_index, upper_index) += R_recomb * sr;
            at(coll_bf, upper_index, upper_index) -= C_recomb * sr;
            at(coll_bf, lower_index, upper_index) += C_recomb * sr;
          }
        }
      }
      if (c.rp.nt_on) {
        // nltepop.cc:564-591 nltepop_matrix_add_nt_ionisation
        const double Y_nt = r.g->ntY[nix(c, mgi, e, i)];
        for (int upperion = i + 1; upperion <= nt_ionisation_maxupperion(c, e, i); upperion++) {
          const double Y_nt_thisupperion = Y_nt * nt_ionization_upperion_probability(c, mgi, e, i, upperion, false);
          if (Y_nt_thisupperion > 0.) {
            const int upper_groundstate_index = nlte_vector_index(c, e, upperion, 0);
            for (int level = 0; level < nlevels; level++) {
              const int lower_index = nlte_vector_index(c, e, i, level);
              at(ntcoll_bf, lower_index, lower_index) -= Y_nt_thisupperion * s_renorm[level];
              at(ntcoll_bf, upper_groundstate_index, lower_index) += Y_nt_thisupperion * s_renorm[level];
            }
          }
        }
      }
    }
  }
  A.assign((size_t)D * D, 0.);
  for (size_t q = 0; q < A.size(); q++) A[q] = ((((A[q] + rad_bb[q]) + coll_bb[q]) + rad_bf[q]) + coll_bf[q]) + ntcoll_bf[q];
  if (getenv("ORACLE_NL_DUMP")) tl_raw_matrix = A;  // diagnostics: the rate matrix before normalisation
  for (int col = 0; col < D; col++) A[(size_t)col * D + 0] = 1.0;  // normalisation row
  b.assign(D, 0.);
  b[0] = nl_elem_numberdens(c, r, mgi, e);
  // nltepop.cc:593-628 nltepop_matrix_normalise
  norm.assign(D, 0.);
  for (int col = 0; col < D; col++) {
    int ion = 0, level = 0;
    nlte_ion_level_of_index(c, col, e, &ion, &level);
    norm[col] = calculate_levelpop_lte(c, mgi, e, ion, level);
    if (level != 0 && !is_nlte(c, e, ion, level)) {
      for (int dl = level + 1; dl < get_nlevels(c, e, ion); dl++)
        if (!is_nlte(c, e, ion, dl)) norm[col] += calculate_levelpop_lte(c, mgi, e, ion, dl);
    }
    for (int row = 0; row < D; row++) A[(size_t)col * D + row] *= norm[col];
  }
  return D;
}
// nltepop.cc:798-1113 solve_nlte_pops_element; -1 on the reference's assert_always aborts
int nl_solve_nlte_pops_element(const Ctx &c, const NlteRun &r, int e, int mgi, std::vector<double> *A_out) {
  if (r.in->elem_abundance[(size_t)mgi * c.at->nelements + e] <= 0.) {
    nlte_reset_element(c, r, mgi, e);
    return 0;
  }
  std::vector<double> A, b, norm, slpf;
  const int D = nlte_build(c, r, mgi, e, A, b, norm, slpf);
  if (A_out) *A_out = A;
  std::vector<double> popvec(D);
  const bool solved = nlte_matrix_solve(A.data(), b.data(), D, popvec.data(), norm.data());
  if (const char *dump = getenv("ORACLE_NL_DUMP")) {
    // diagnostics: the first solve of each element (tools/nl_dump_cmp.py)
    static int ncalls[64] = {0};  // solves of each element so far under this prefix (a one-cell diagnostic run)
    static std::string last;
    if (last != dump) {
      last = dump;
      for (int q = 0; q < 64; q++) ncalls[q] = 0;
    }
    const int pass = e < 64 ? ncalls[e]++ : 99;
    const std::string path = std::string(dump) + "_p" + std::to_string(pass) + "_ora_e" + std::to_string(e) + ".bin";
    if (pass < 4) if (FILE *fp = fopen(path.c_str(), "wb")) {
      const int32_t hdr[2] = {D, solved ? 0 : 1};
      fwrite(hdr, sizeof hdr, 1, fp);
      fwrite(A.data(), 8, A.size(), fp);
      fwrite(b.data(), 8, b.size(), fp);
      fwrite(norm.data(), 8, norm.size(), fp);
      fwrite(popvec.data(), 8, popvec.size(), fp);
      fwrite(tl_raw_matrix.data(), 8, tl_raw_matrix.size(), fp);
      fclose(fp);
    }
  }
  if (!solved) {
    nlte_reset_element(c, r, mgi, e);  // set_element_pops_lte
    return 0;
  }
  for (int k = 0; k < D; k++)
    if (!std::isfinite(popvec[k]) || !(popvec[k] >= 0.)) {
      if (getenv("ORACLE_DEBUG")) {
        fprintf(stderr, "oracle nlte: element %d D %d popvec[%d] = %g norm %g b0 %g\n", e, D, k, popvec[k], norm[k], b[0]);
        for (int q = 0; q < D; q++) fprintf(stderr, "  norm[%d] %g pop %g A[q][q] %g\n", q, norm[q], popvec[q], A[(size_t)q * D + q]);
      }
      return -1;
    }
  double *row = r.g->nlte_pops.data() + (size_t)mgi * c.at->total_nlte_levels;
  const double rho = r.in->rho[mgi];
  for (int i = 0; i < get_nions(c, e); i++) {
    const int nn = get_nlevels_nlte(c, e, i);
    const int index_gs = nlte_vector_index(c, e, i, 0);
    const int nlte_start = c.at->ion_first_nlte[uion(c, e, i)];
    for (int level = 1; level <= nn; level++) row[nlte_start + level - 1] = popvec[nlte_vector_index(c, e, i, level)] / rho;
    if (ion_has_superlevel(c, e, i))
      row[nlte_start + nn] = (popvec[nlte_vector_index(c, e, i, nn + 1)] / rho / slpf[i]);
    nl_gp(c, r, mgi, e, i) = popvec[index_gs];
  }
  double elem_pop_matrix = 0.;  // gsl_blas_dasum
  for (int k = 0; k < D; k++) elem_pop_matrix += fabs(popvec[k]);
  const double elem_pop_abundance = nl_elem_numberdens(c, r, mgi, e);
  const double elem_pop_error_percent = fabs((elem_pop_abundance / elem_pop_matrix) - 1) * 100;
  if (elem_pop_error_percent > 1.0) nlte_reset_element(c, r, mgi, e);
  return 0;
}

// kpkt.cc:84-165 calculate_cooling_rates into the caller's arrays
void nl_store_cooling(const Ctx &c, const NlteRun &r, int mgi) {
  te_calculate_cooling_rates(c, mgi, nullptr, &r.in->totalcooling[mgi],
                             r.in->cooling_contrib_ion + (size_t)mgi * c.at->nions_total);
}

}  // namespace

extern "C" {
// artis_gpu_update_grid_nlte restated (include/artis_gpu.h): the listed cells in parallel (OpenMP), each in the
// reference's serial order.  Returns ARTIS_ERR_PACKET_FAULT when a cell hits one of the reference's abort paths.
int oracle_update_grid_nlte(const artis_atomic_tables *at, const artis_run_params *rp, const artis_nt_shells *nt,
                            const artis_nlte_params *p, artis_nlte_cells *in, int npts_model, int nthreads) {
  if (!rp->nlte_pops_on || !rp->no_lut_photoion || !rp->no_lut_bfheating || !rp->multibin_radfield) return ARTIS_ERR_UNSUPPORTED;
  const size_t ni = at->nions_total, nb = at->radfield_nbins, nbf = at->nbfcontinua;
  const size_t A1 = kNtMaxAuger + 1;
  NlteGrid g;
  g.Te.assign(in->Te, in->Te + npts_model);
  g.TR.assign(in->TR, in->TR + npts_model);
  g.W.assign(in->W, in->W + npts_model);
  g.TJ.assign(in->TJ, in->TJ + npts_model);
  g.nne.assign(in->nne, in->nne + npts_model);
  g.nnetot.assign(in->nnetot, in->nnetot + npts_model);
  g.gp.assign(in->groundlevelpop, in->groundlevelpop + (size_t)npts_model * ni);
  g.pf.assign(in->partfunct, in->partfunct + (size_t)npts_model * ni);
  g.binTR.assign(in->bin_TR, in->bin_TR + (size_t)npts_model * nb);
  g.binW.assign(in->bin_W, in->bin_W + (size_t)npts_model * nb);
  g.bfrate.assign(in->bfrate_estimator, in->bfrate_estimator + (size_t)npts_model * nbf);
  g.nlte_pops.assign(in->nlte_pops, in->nlte_pops + (size_t)npts_model * at->total_nlte_levels);
  g.ntY.assign((size_t)npts_model * ni, 0.);
  g.nt_prob.assign(in->nt_prob_num_auger, in->nt_prob_num_auger + (size_t)npts_model * ni * A1);
  g.nt_ionen.assign(in->nt_ionenfrac_num_auger, in->nt_ionenfrac_num_auger + (size_t)npts_model * ni * A1);
  artis_cell_state cs;
  memset(&cs, 0, sizeof(cs));
  cs.Te = g.Te.data();
  cs.TR = g.TR.data();
  cs.TJ = g.TJ.data();
  cs.W = g.W.data();
  cs.nne = g.nne.data();
  cs.nnetot = g.nnetot.data();
  cs.rho = in->rho;
  cs.elem_abundance = in->elem_abundance;
  cs.groundlevelpop = g.gp.data();
  cs.partfunct = g.pf.data();
  cs.nlte_pops = g.nlte_pops.data();
  cs.radfield_bin_TR = g.binTR.data();
  cs.radfield_bin_W = g.binW.data();
  cs.bfrate_estimator = g.bfrate.data();
  cs.nt_deposition_rate_density = in->deposition_rate_density;
  cs.nt_ionization_ratecoeff = g.ntY.data();
  cs.nt_prob_num_auger = g.nt_prob.data();
  cs.nt_ionenfrac_num_auger = g.nt_ionen.data();
  Ctx c;
  c.at = at;
  c.g = nullptr;
  c.cs = &cs;
  c.rp = *rp;
  c.gs = nullptr;
  c.T_step_log = (log(at->maxtemp) - log(at->mintemp)) / (at->tablesize - 1.);
  c.minpop = rp->minpop > 0. ? rp->minpop : 1e-30;
  c.nts = p->nts;
  {
    int64_t ntg = 0;
    for (int lv = 0; lv < at->nlevels_total; lv++) ntg += at->level_nphixstargets[lv];
    c.slot_allcont.assign(ntg + 1, -1);
    for (int ib = 0; ib < at->nbfcontinua; ib++) {
      const int ul = at->ion_uniqueleveloffset[at->elem_uniqueionoffset[at->allcont_element[ib]] + at->allcont_ion[ib]] +
                     at->allcont_level[ib];
      c.slot_allcont[at->level_phixstargets_offset[ul] + at->allcont_phixstargetindex[ib]] = ib;
    }
  }
  NlteRun r{p, nt, in, &g, SfGrid()};
  if (rp->nt_on && rp->nt_solve_spencerfano) sf_setup(r.sf, nt);
  int rc = 0;
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic)
  for (int k = 0; k < in->ncells; k++) {
    const int mgi = in->mgi[k];
    int fail = 0;
    int iters = 0;
    TeRates hc;
    memset(&hc, 0, sizeof(hc));
    const double deltaV = in->vol_init[mgi] * pow(p->tratmid, 3);
    const double estimator_normfactor = 1 / deltaV / p->deltat / p->nprocs;
    const double estimator_normfactor_over4pi = ARTIS_ONEOVER4PI * estimator_normfactor;
    const double J = in->J[mgi] * estimator_normfactor_over4pi;  // radfield::normalise_J
    if (p->initial_iteration || in->thick[mgi] == 1) {
      // update_grid.cc:1106-1125
      double T_J = pow(J * ARTIS_PI / ARTIS_STEBO, 1. / 4.);
      if (!std::isfinite(T_J))
        T_J = g.TR[mgi];
      else if (T_J > p->T_max)
        T_J = p->T_max;
      else if (T_J < p->T_min)
        T_J = p->T_min;
      g.TR[mgi] = T_J;
      g.Te[mgi] = T_J;
      g.TJ[mgi] = T_J;
      g.W[mgi] = 1;
      nl_precalculate_partfuncts(c, r, mgi);
      if (nl_calculate_populations_lte(c, r, mgi) != 0) fail = 1;
    } else {
      // update_grid.cc:1126-1154
      const double nuJ = in->nuJ[mgi] * estimator_normfactor_over4pi;
      const double ffheat = in->ffheating[mgi] * estimator_normfactor;
      nl_fit_parameters(c, r, mgi, J, nuJ, estimator_normfactor_over4pi, &fail);
      for (size_t q = 0; q < nbf; q++)  // normalise_bf_estimators (estimator_normfactor / H)
        g.bfrate[(size_t)mgi * nbf + q] = in->bfrate_raw[(size_t)mgi * nbf + q] * (estimator_normfactor / ARTIS_H);
      // update_grid.cc:763-886 solve_Te_nltepops
      std::vector<double> coeff;
      if (nl_calculate_bfheatingcoeffs(c, r, mgi, coeff) != 0) fail = 1;
      for (int nlte_iter = 0; nlte_iter <= p->nlteiter && !fail; nlte_iter++) {
        iters = nlte_iter + 1;
        if (rp->nt_on && rp->nt_solve_spencerfano) nl_solve_spencerfano(c, r, mgi, p->nts, &fail, nullptr);
        if (rp->nt_on) nl_store_nt_rates(c, r, mgi, &fail);
        const double prev_T_e = g.Te[mgi];
        if (nl_call_T_e_finder(c, r, mgi, coeff, ffheat, &hc) != 0) {
          fail = 1;
          if (getenv("ORACLE_DEBUG")) fprintf(stderr, "oracle nlte: cell %d iter %d T_e finder GSL abort\n", mgi, nlte_iter);
        }
        const double fracdiff_T_e = fabs((g.Te[mgi] / prev_T_e) - 1);
        for (int e = 0; e < at->nelements && !fail; e++)
          if (get_nions(c, e) > 0 && nl_solve_nlte_pops_element(c, r, e, mgi, nullptr) != 0) {
            fail = 1;
            if (getenv("ORACLE_DEBUG")) fprintf(stderr, "oracle nlte: cell %d iter %d element %d bad populations\n", mgi, nlte_iter, e);
          }
        const double nne_prev = g.nne[mgi];
        nl_precalculate_partfuncts(c, r, mgi);
        nl_calculate_electron_densities(c, r, mgi);
        const double fracdiff_nne = fabs((g.nne[mgi] / nne_prev) - 1);
        if (fracdiff_nne <= 0.04 && fracdiff_T_e <= 0.04) break;
      }
    }
    if (fail) {
#pragma omp critical
      rc = ARTIS_ERR_PACKET_FAULT;
      continue;
    }
    if (rp->nt_on) nl_store_nt_rates(c, r, mgi, &fail);
    nl_store_cooling(c, r, mgi);
    in->Te[mgi] = g.Te[mgi];
    in->TR[mgi] = g.TR[mgi];
    in->W[mgi] = g.W[mgi];
    in->TJ[mgi] = g.TJ[mgi];
    in->nne[mgi] = g.nne[mgi];
    in->nnetot[mgi] = g.nnetot[mgi];
    for (size_t u = 0; u < ni; u++) {
      in->groundlevelpop[(size_t)mgi * ni + u] = g.gp[(size_t)mgi * ni + u];
      in->partfunct[(size_t)mgi * ni + u] = g.pf[(size_t)mgi * ni + u];
      in->nt_ionization_ratecoeff[(size_t)mgi * ni + u] = g.ntY[(size_t)mgi * ni + u];
    }
    for (size_t q = 0; q < ni * A1; q++) {
      in->nt_prob_num_auger[(size_t)mgi * ni * A1 + q] = g.nt_prob[(size_t)mgi * ni * A1 + q];
      in->nt_ionenfrac_num_auger[(size_t)mgi * ni * A1 + q] = g.nt_ionen[(size_t)mgi * ni * A1 + q];
    }
    for (size_t q = 0; q < nb; q++) {
      in->bin_TR[(size_t)mgi * nb + q] = g.binTR[(size_t)mgi * nb + q];
      in->bin_W[(size_t)mgi * nb + q] = g.binW[(size_t)mgi * nb + q];
    }
    for (size_t q = 0; q < nbf; q++) in->bfrate_estimator[(size_t)mgi * nbf + q] = g.bfrate[(size_t)mgi * nbf + q];
    for (int q = 0; q < at->total_nlte_levels; q++)
      in->nlte_pops[(size_t)mgi * at->total_nlte_levels + q] = g.nlte_pops[(size_t)mgi * at->total_nlte_levels + q];
    if (in->heatingcoolingrates) memcpy(in->heatingcoolingrates + (size_t)mgi * ARTIS_TE_NRATES, &hc, sizeof(hc));
    if (in->nlte_iterations) in->nlte_iterations[mgi] = iters;
  }
  return rc;
}

// ---- pins of the restated numerical kernels (tests/test_nebular_update_grid.py) ----
// nltepop_matrix_solve (LU with partial pivoting, refinement, D11) on a column-major n x n system, unit
// normalisation; returns 1 if singular
int oracle_nl_matrix_solve(const double *A, const double *b, int n, double *x) {
  std::vector<double> norm(n, 1.);
  return nlte_matrix_solve(A, b, n, x, norm.data()) ? 0 : 1;
}
// sfmatrix_solve on a row-major upper-triangular n x n system
void oracle_sf_solve(const double *U, const double *b, int n, double *y) { sf_solve(U, b, n, y); }
// radfield.cc planck_integral (GSL qag restated, epsrel 1e-10)
double oracle_planck_integral(double T_R, double nu_lower, double nu_upper, int times_nu) {
  return nl_planck_integral(T_R, nu_lower, nu_upper, times_nu != 0);
}
// the Spencer-Fano energy grid, source and loss terms: envec, sourcevec, the right-hand side and the loss diagonal
// for an electron density nne; returns E_init_ev
double oracle_sf_grid(int sfpts, double emin, double emax, double nne, double *envec, double *sourcevec, double *rhs,
                      double *loss_diag) {
  artis_nt_shells nt;
  memset(&nt, 0, sizeof(nt));
  nt.sfpts = sfpts;
  nt.sf_emin = emin;
  nt.sf_emax = emax;
  SfGrid g;
  sf_setup(g, &nt);
  for (int i = 0; i < g.n; i++) {
    envec[i] = g.envec[i];
    sourcevec[i] = g.sourcevec[i];
    double dasum = 0.;
    if (i < g.n - 1)
      for (int j = i + 1; j < g.n; j++) dasum += fabs(g.sourcevec[j]);
    rhs[i] = (i < g.n - 1) ? dasum * g.delta_e : 0.;
    loss_diag[i] = sf_electron_loss_rate(g.envec[i] * ARTIS_EV, nne) / ARTIS_EV;
  }
  return g.E_init_ev;
}
}  // extern "C"
