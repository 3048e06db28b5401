// te_solver.h -- update_grid's temperature / ionisation solution on the GPU for the LTE-population options
// (artis_gpu_solve_temperatures, include/artis_gpu.h).
//
// One model cell per workitem, each running the reference's serial algorithm in the reference's operation order
// (so the results are the oracle's bit for bit): the lanes of a wave are 64 cells that walk the same atomic data
// (level lists, line lists, LUT rows) in lockstep, so every table load is wave-uniform and the FP64 work --
// dominated by the collisional-excitation cooling over all lines in every thermal-balance evaluation
// (kpkt.cc:41-67) -- runs on all 64 lanes.  Divergence is confined to the Brent iteration counts.
//
//   k_te_bfheat   calculate_bfheatingcoeffs (thermalbalance.cc:141-187, LUT branch) for the ionising levels the
//                 heating sum visits, per cell into a cell-minor scratch
//   k_te_solve    precalculate_partfuncts, call_T_e_finder (GSL Brent on T_e_eqn_heating_minus_cooling, each
//                 evaluation solving calculate_populations with its own Brent on n_e), the final
//                 calculate_populations and calculate_cooling_rates; or the LTE branch (update_grid.cc:1106-1125)
#pragma once

struct TeDev {
  // tables
  const double *bfheat_lut;  // [tablesize * nbf]
  const float *alpha_sp;     // [nions_total * tablesize]
  const int32_t *anumber;    // [nelements]
  const int32_t *hb_ul;      // [nhb] ionising levels of every ion but the top one, calculate_heating_rates' order
  int32_t nhb;
  int32_t ncells;
  const int32_t *mgi;  // [ncells]
  // parameters
  double t_current, tmin, T_min, T_max, accuracy;
  int32_t initial_iteration;
  // inputs by mgi
  const float *TR, *W, *TJ, *rho, *abund, *meanw;
  const int16_t *thick;
  const double *vol, *ffheat, *colheat, *gamma, *bfest, *hdep;
  // in / out by mgi
  float *Te, *gp;
  // outputs by mgi
  float *nne, *nnetot, *pf;
  double *totcool, *ccion, *rates;
  int32_t *iters;
  // scratch: uppermost ion [mgi * nelements + e], bf-heating coefficients [j * ncells + k]
  int32_t *upp;
  double *hbc;
  int32_t *fail;  // first failing cell (mgi + 1): the reference's GSL abort paths
  // DIRECT_COL_HEAT: the collisional heating is the de-excitation sum (thermalbalance.cc:189-238)
  int32_t direct_col_heat;
  // the nebular solution (nlte_solver.h): NLTE / superlevel populations by mgi (ltepop.cc:349-415; nullptr: LTE
  // populations), and the mode of k_te_solve: 0 the full solution above, 1 only call_T_e_finder with
  // calculate_electron_densities (NLTE_POPS_ALL_IONS_SIMULTANEOUS, thermalbalance.cc:357-361), 2 only the final
  // calculate_cooling_rates
  const double *nlte;
  int32_t mode;
  // row of a cell's bf-heating coefficients in hbc: hbk[k] (nullptr: k) of hbstride rows
  const int32_t *hbk;
  int32_t hbstride;
};

struct TeState {
  int k, mgi;
  float Te;
  int g, sub, lane0;  // the cell's lane group: size, this lane's index in it, its first lane in the wave
  double *phi;        // [nions_total] in LDS: phi of the ions below each element's uppermost ion (one per cell;
                      // the group's lanes store identical values)
};

// ltepop.cc:307-327
DEVFN double te_get_gp(const Ctx &K, const TeDev &D, int mgi, int ui, int e) {
  const double nn = D.gp[(int64_t)mgi * K.T.nions_total + ui];
  if (nn < K.R.minpop) {
    if (D.abund[(int64_t)mgi * K.T.nelements + e] > 0) return K.R.minpop;
    return 0.;
  }
  return nn;
}
// ltepop.cc:349-415 with NLTE_POPS_ON: an NLTE level's (or the superlevel's, nltepop.cc:1543-1554) stored population
// when there is one (not < -0.9); returns false for the LTE expression
DEVFN bool te_nlte_levelpop(const Ctx &K, const TeDev &D, const TeState &s, int ui, int l, double *nn) {
  if (!D.nlte || l == 0) return false;
  const int nn_nlte = K.T.ion_nlevels_nlte[ui];
  const double *row = D.nlte + (int64_t)s.mgi * K.T.total_nlte_levels + K.T.ion_first_nlte[ui];
  const double rho = D.rho[s.mgi];
  if (l <= nn_nlte) {
    const double v = row[l - 1];
    if (v < -0.9) return false;
    *nn = v * rho;
    return true;
  }
  const double v = row[nn_nlte];
  if (v < -0.9) return false;
  const int ul0 = K.T.ion_uniqueleveloffset[ui];
  const int sl = ul0 + nn_nlte + 1;
  const double T_exc = K.R.exc_te ? (double)s.Te : (double)D.TJ[s.mgi];
  const double boltz = (double)K.T.level_stat_weight[ul0 + l] / (double)K.T.level_stat_weight[sl] *
                       exp(-(K.T.level_epsilon[ul0 + l] - K.T.level_epsilon[sl]) / ARTIS_KB / T_exc);
  *nn = v * rho * boltz;
  return true;
}
// ltepop.cc:329-347, 349-415
DEVFN double te_levelpop_nominpop(const Ctx &K, const TeDev &D, const TeState &s, int e, int ui, int l) {
  const double nnground = te_get_gp(K, D, s.mgi, ui, e);
  if (l == 0) return nnground;
  double nlte;
  if (te_nlte_levelpop(K, D, s, ui, l, &nlte)) return nlte;
  const double T_exc = K.R.exc_te ? (double)s.Te : (double)D.TJ[s.mgi];
  const double W = 1.;
  const int ul0 = K.T.ion_uniqueleveloffset[ui];
  const double E_level = K.T.level_epsilon[ul0 + l];
  const double E_ground = K.T.level_epsilon[ul0];
  return (nnground * W * (double)K.T.level_stat_weight[ul0 + l] / (double)K.T.level_stat_weight[ul0] *
          exp(-(E_level - E_ground) / ARTIS_KB / T_exc));
}
// ltepop.cc:417-430
DEVFN double te_levelpop(const Ctx &K, const TeDev &D, const TeState &s, int e, int ui, int l) {
  double nn;
  if (te_nlte_levelpop(K, D, s, ui, l, &nn)) return nn;  // skipminpop
  nn = te_levelpop_nominpop(K, D, s, e, ui, l);
  if (nn < K.R.minpop) nn = (D.abund[(int64_t)s.mgi * K.T.nelements + e] > 0) ? K.R.minpop : 0.;
  return nn;
}
// ltepop.cc:558-564
DEVFN double te_ionstagepop(const Ctx &K, const TeDev &D, const TeState &s, int e, int ui) {
  return te_get_gp(K, D, s.mgi, ui, e) * D.pf[(int64_t)s.mgi * K.T.nions_total + ui] /
         (double)K.T.level_stat_weight[K.T.ion_uniqueleveloffset[ui]];
}

// ltepop.cc:488-537 + update_grid.cc:23-38
DEVNI void te_precalculate_partfuncts(const Ctx &K, const TeDev &D, const TeState &s) {
  const int ni = K.T.nions_total;
  for (int e = 0; e < K.T.nelements; e++)
    for (int i = 0; i < K.T.elem_nions[e]; i++) {
      const int ui = uion(K, e, i);
      float &gpref = D.gp[(int64_t)s.mgi * ni + ui];
      int initial = 0;
      double pop_store = 0.;
      if (te_get_gp(K, D, s.mgi, ui, e) < K.R.minpop) {
        pop_store = te_get_gp(K, D, s.mgi, ui, e);
        initial = 1;
        gpref = 1.0f;
      }
      double U = 1.;
      const int nlevels = K.T.ion_nlevels[ui];
      const double groundpop = te_get_gp(K, D, s.mgi, ui, e);
      for (int level = 1; level < nlevels; level++) U += te_levelpop_nominpop(K, D, s, e, ui, level) / groundpop;
      U *= (double)K.T.level_stat_weight[K.T.ion_uniqueleveloffset[ui]];
      if (initial == 1) gpref = pop_store;
      D.pf[(int64_t)s.mgi * ni + ui] = U;
    }
}

// GSL roots/brent.c, roots/convergence.c (see oracle.cc): status -1 = the GSL_ERROR (abort) paths
struct TeBrent {
  double a, b, c, d, e, fa, fb, fc, root, x_lower, x_upper;
};
template <class F>
DEVFN int te_brent_set(TeBrent &s, F &f, double x_lower, double x_upper) {
  s.root = 0.5 * (x_lower + x_upper);
  s.x_lower = x_lower;
  s.x_upper = x_upper;
  const double f_lower = f(x_lower);
  if (!isfinite(f_lower)) return -1;
  const double f_upper = f(x_upper);
  if (!isfinite(f_upper)) return -1;
  s.a = x_lower;
  s.fa = f_lower;
  s.b = x_upper;
  s.fb = f_upper;
  s.c = x_upper;
  s.fc = f_upper;
  s.d = x_upper - x_lower;
  s.e = x_upper - x_lower;
  if ((f_lower < 0.0 && f_upper < 0.0) || (f_lower > 0.0 && f_upper > 0.0)) return -1;
  return 0;
}
template <class F>
DEVFN int te_brent_iterate(TeBrent &s, F &f) {
  double a = s.a, b = s.b, c = s.c, fa = s.fa, fb = s.fb, fc = s.fc, d = s.d, e = s.e;
  int ac_equal = 0;
  if ((fb < 0 && fc < 0) || (fb > 0 && fc > 0)) {
    ac_equal = 1;
    c = a;
    fc = fa;
    d = b - a;
    e = b - a;
  }
  if (fabs(fc) < fabs(fb)) {
    ac_equal = 1;
    a = b;
    b = c;
    c = a;
    fa = fb;
    fb = fc;
    fc = fa;
  }
  const double tol = 0.5 * DBL_EPSILON * fabs(b);
  const double m = 0.5 * (c - b);
  if (fb == 0) {
    s.root = b;
    s.x_lower = b;
    s.x_upper = b;
    return 0;
  }
  if (fabs(m) <= tol) {
    s.root = b;
    if (b < c) {
      s.x_lower = b;
      s.x_upper = c;
    } else {
      s.x_lower = c;
      s.x_upper = b;
    }
    return 0;
  }
  if (fabs(e) < tol || fabs(fa) <= fabs(fb)) {
    d = m;
    e = m;
  } else {
    double p, q, r;
    const double sr = fb / fa;
    if (ac_equal) {
      p = 2 * m * sr;
      q = 1 - sr;
    } else {
      q = fa / fc;
      r = fb / fc;
      p = sr * (2 * m * q * (q - r) - (b - a) * (r - 1));
      q = (q - 1) * (r - 1) * (sr - 1);
    }
    if (p > 0)
      q = -q;
    else
      p = -p;
    if (2 * p < fmin(3 * m * q - fabs(tol * q), fabs(e * q))) {
      e = d;
      d = p / q;
    } else {
      d = m;
      e = m;
    }
  }
  a = b;
  fa = fb;
  if (fabs(d) > tol)
    b += d;
  else
    b += (m > 0 ? +tol : -tol);
  fb = f(b);
  if (!isfinite(fb)) return -1;
  s.a = a;
  s.b = b;
  s.c = c;
  s.d = d;
  s.e = e;
  s.fa = fa;
  s.fb = fb;
  s.fc = fc;
  s.root = b;
  if ((fb < 0 && fc < 0) || (fb > 0 && fc > 0)) c = a;
  if (b < c) {
    s.x_lower = b;
    s.x_upper = c;
  } else {
    s.x_lower = c;
    s.x_upper = b;
  }
  return 0;
}
DEVFN int te_test_interval(double x_lower, double x_upper, double epsabs, double epsrel) {
  const double abs_lower = fabs(x_lower), abs_upper = fabs(x_upper);
  double min_abs;
  if ((x_lower > 0.0 && x_upper > 0.0) || (x_lower < 0.0 && x_upper < 0.0))
    min_abs = fmin(abs_lower, abs_upper);
  else
    min_abs = 0;
  const double tolerance = epsabs + epsrel * min_abs;
  return fabs(x_upper - x_lower) < tolerance ? 0 : 1;
}

DEVFN bool te_use_lte_ratio(const TeDev &D, int mgi) { return D.initial_iteration || D.thick[mgi] == 1; }
// ltepop.cc:97-113
DEVFN double te_ion_alpha_sp(const Ctx &K, const TeDev &D, int ui, double T) {
  const float *alpha = D.alpha_sp + (int64_t)ui * K.T.tablesize;
  const int lowerindex = floor(log(T / K.T.mintemp) / K.T.T_step_log);
  if (lowerindex < K.T.tablesize - 1) {
    const int upperindex = lowerindex + 1;
    const double T_lower = K.T.mintemp * exp(lowerindex * K.T.T_step_log);
    const double T_upper = K.T.mintemp * exp(upperindex * K.T.T_step_log);
    const double f_upper = alpha[upperindex];
    const double f_lower = alpha[lowerindex];
    return f_lower + (f_upper - f_lower) / (T_upper - T_lower) * (T - T_lower);
  }
  return alpha[K.T.tablesize - 1];
}
// ltepop.cc:115-239 (NT_ON false)
DEVFN double te_phi(const Ctx &K, const TeDev &D, const TeState &s, int e, int i) {
  double phi = 0;
  const float T_e = s.Te;
  const int ui = uion(K, e, i);
  const int64_t pfrow = (int64_t)s.mgi * K.T.nions_total;
  if (te_use_lte_ratio(D, s.mgi)) {
    const double ionpot = K.T.level_epsilon[K.T.ion_uniqueleveloffset[ui + 1]] - K.T.level_epsilon[K.T.ion_uniqueleveloffset[ui]];
    const double partfunct_ratio = D.pf[pfrow + ui] / D.pf[pfrow + ui + 1];
    phi = partfunct_ratio * ARTIS_SAHACONST * pow((double)T_e, -1.5) * exp(ionpot / ARTIS_KB / T_e);
  } else {
    const double Gamma = D.gamma[(int64_t)s.mgi * K.T.nelements * K.T.maxnions + e * K.T.maxnions + i];
    const double Gamma_ion = Gamma * (double)K.T.level_stat_weight[K.T.ion_uniqueleveloffset[ui]] / D.pf[pfrow + ui];
    const double Alpha_st = 0.;
    const double Alpha_sp = te_ion_alpha_sp(K, D, ui, T_e);
    const double Col_rec = 0.;
    const double Y_nt = 0.0;
    phi = (Alpha_sp + Alpha_st + Col_rec) / (Gamma_ion + Y_nt);
  }
  return phi;
}
#define TE_MAX_IONS_PER_ELEMENT 32
// ltepop.cc:61-95 get_ionfractions without its arrays: the denominator runs down from the uppermost ion as in the
// reference, and each ion's factor nnionfactor[ion] = nnionfactor[ion + 1] * nne * phi is rebuilt by the same chain
// of products (identical bits; the chains are a few ions long).  phi of every ion below the uppermost one is the value
// te_calculate_populations stored for this T_e (the reference recomputes the same pure function).
DEVFN double te_ionfrac_denominator(const double *phi, int ui0, int uppermost_ion, double nne) {
  double f = 1., denominator = 1.;
  for (int ion = uppermost_ion - 1; ion >= 0; ion--) {
    f = f * nne * phi[ui0 + ion];
    denominator += f;
  }
  return denominator;
}
DEVFN double te_ionfraction(const double *phi, int ui0, int uppermost_ion, double nne, double denominator, int ion) {
  double numerator = 1.;
  for (int j = uppermost_ion - 1; j >= ion; j--) numerator = numerator * nne * phi[ui0 + j];
  double fr = numerator / denominator;
  if (!isfinite(fr)) fr = 0;
  return fr;
}
DEVFN double te_elem_numberdens(const Ctx &K, const TeDev &D, int mgi, int e) {
  const double mw = D.meanw[(int64_t)mgi * K.T.nelements + e];
  return D.abund[(int64_t)mgi * K.T.nelements + e] / mw * (double)D.rho[mgi];
}
// ltepop.cc:20-59
DEVNI double te_nne_solution_f(const Ctx &K, const TeDev &D, const TeState &s, double x) {
  const double rho = D.rho[s.mgi];
  double outersum = 0.;
  for (int e = 0; e < K.T.nelements; e++) {
    const float abundance = D.abund[(int64_t)s.mgi * K.T.nelements + e];
    if (abundance > 0 && K.T.elem_nions[e] > 0) {
      const double elem_mw = D.meanw[(int64_t)s.mgi * K.T.nelements + e];
      double innersum = 0.;
      const int uppermost_ion = D.upp[(int64_t)s.mgi * K.T.nelements + e];
      const int ui0 = K.T.elem_uniqueionoffset[e];
      const double den = te_ionfrac_denominator(s.phi, ui0, uppermost_ion, x);
      for (int ion = 0; ion <= uppermost_ion; ion++)
        innersum += (get_ionstage(K, e, ion) - 1) * te_ionfraction(s.phi, ui0, uppermost_ion, x, den, ion);
      outersum += abundance / elem_mw * innersum;
    }
  }
  return rho * outersum - x;
}
// update_grid.cc:1427-1658 (NO_LUT_PHOTOION false, NT_ON false); -1: the GSL abort path
DEVNI int te_calculate_populations(const Ctx &K, const TeDev &D, const TeState &s, double *nntot_out) {
  const int nel = K.T.nelements, ni = K.T.nions_total;
  const int mgi = s.mgi;
  double nne_hi = D.rho[mgi] / ARTIS_MH;
  int only_neutral_ions = 0;
  int nelements_in_cell = 0;
  for (int e = 0; e < nel; e++) {
    const int nions = K.T.elem_nions[e];
    int32_t *upp = &D.upp[(int64_t)mgi * nel + e];
    *upp = nions - 1;
    const double abundance = D.abund[(int64_t)mgi * nel + e];
    if (abundance > 0) {
      int uppermost_ion;
      if (te_use_lte_ratio(D, mgi)) {
        uppermost_ion = nions - 1;
      } else {
        int ion;
        for (ion = 0; ion < nions - 1; ion++) {
          const double Gamma = D.gamma[(int64_t)mgi * nel * K.T.maxnions + e * K.T.maxnions + ion];
          if (Gamma == 0) break;
        }
        uppermost_ion = ion;
      }
      double factor = 1.;
      int ion;
      for (ion = 0; ion < uppermost_ion; ion++) {
        const double phi = te_phi(K, D, s, e, ion);
        s.phi[uion(K, e, ion)] = phi;
        factor *= nne_hi * phi;
        if (!isfinite(factor)) break;
      }
      uppermost_ion = ion;
      *upp = uppermost_ion;
      if (uppermost_ion == 0) only_neutral_ions++;
      nelements_in_cell++;
    }
  }
  float nne = 0.;
  double nne_tot = 0.;
  double nntot = 0.;
  if (only_neutral_ions == nelements_in_cell) {
    for (int e = 0; e < nel; e++) {
      const double nnelement = te_elem_numberdens(K, D, mgi, e);
      nne_tot += nnelement * D.anumber[e];
      const int nions = K.T.elem_nions[e];
      for (int ion = 0; ion < nions; ion++) {
        double nnion;
        if (ion == 0)
          nnion = nnelement;
        else if (nnelement > 0.)
          nnion = K.R.minpop;
        else
          nnion = 0.;
        nntot += nnion;
        nne += nnion * (get_ionstage(K, e, ion) - 1);
        const int ui = uion(K, e, ion);
        D.gp[(int64_t)mgi * ni + ui] =
            (nnion * (double)K.T.level_stat_weight[K.T.ion_uniqueleveloffset[ui]] / D.pf[(int64_t)mgi * ni + ui]);
      }
    }
    nntot += nne;
    if (nne < K.R.minpop) nne = K.R.minpop;
    D.nne[mgi] = nne;
  } else {
    double nne_lo = 0.;
    auto f = [&](double x) { return te_nne_solution_f(K, D, s, x); };
    TeBrent b;
    if (te_brent_set(b, f, nne_lo, nne_hi) != 0) return -1;
    int iter = 0;
    const int maxit = 100;
    const double fractional_accuracy = 1e-3;
    int status;
    do {
      iter++;
      if (te_brent_iterate(b, f) != 0) return -1;
      nne = b.root;
      nne_lo = b.x_lower;
      nne_hi = b.x_upper;
      status = te_test_interval(nne_lo, nne_hi, 0, fractional_accuracy);
    } while (status == 1 && iter < maxit);
    if (nne < K.R.minpop) nne = K.R.minpop;
    D.nne[mgi] = nne;
    nne_tot = 0.;
    nntot = nne;
    for (int e = 0; e < nel; e++) {
      const int nions = K.T.elem_nions[e];
      const double nnelement = te_elem_numberdens(K, D, mgi, e);
      nne_tot += nnelement * D.anumber[e];
      const int uppermost_ion = D.upp[(int64_t)mgi * nel + e];
      const int ui0 = K.T.elem_uniqueionoffset[e];
      const double den = nnelement > 0 ? te_ionfrac_denominator(s.phi, ui0, uppermost_ion, nne) : 1.;
      for (int ion = 0; ion < nions; ion++) {
        double nnion;
        if (ion <= uppermost_ion) {
          if (nnelement > 0) {
            nnion = nnelement * te_ionfraction(s.phi, ui0, uppermost_ion, nne, den, ion);
            if (nnion < K.R.minpop) nnion = K.R.minpop;
          } else {
            nnion = 0.;
          }
        } else {
          nnion = K.R.minpop;
        }
        nntot += nnion;
        const int ui = uion(K, e, ion);
        D.gp[(int64_t)mgi * ni + ui] =
            (nnion * (double)K.T.level_stat_weight[K.T.ion_uniqueleveloffset[ui]] / D.pf[(int64_t)mgi * ni + ui]);
      }
    }
  }
  D.nnetot[mgi] = nne_tot;
  *nntot_out = nntot;
  return 0;
}

// update_grid.cc:1660-1685 calculate_electron_densities: n_e from the ion-stage populations; returns nne_tot
DEVNI double te_electron_densities(const Ctx &K, const TeDev &D, const TeState &s) {
  double nne_tot = 0.;
  float nne = 0.;
  for (int e = 0; e < K.T.nelements; e++) {
    const double nnelement = te_elem_numberdens(K, D, s.mgi, e);
    nne_tot += nnelement * D.anumber[e];
    if (nnelement > 0)
      for (int i = 0; i < K.T.elem_nions[e]; i++) nne += (get_ionstage(K, e, i) - 1) * te_ionstagepop(K, D, s, e, uion(K, e, i));
  }
  D.nne[s.mgi] = nne;
  D.nnetot[s.mgi] = nne_tot;
  return nne_tot;
}

struct TeRates {
  double cooling_collisional, cooling_fb, cooling_ff, cooling_adiabatic, heating_collisional, heating_bf, heating_ff,
      heating_dep;
};
// (te_col_exc, the exact collisional-excitation term on a packed item: physics.h)
// te_col_exc for k_te_solve, whose lanes are on different ions' lines: one exp -- of +eoverkt or -eoverkt, the
// argument the line's branch takes -- and one log for every lane, instead of the three branches' transcendentals
// run one after another by a divergent wave; the T_e-only factors of the branches evaluated once per sum (TeExcT), the
// divisions by k T_e and by the level's statistical weight made multiplications: the reference's expression up to
// the order of its products (ulp-level differences; update_grid's parity bar is identical Brent iteration counts and T_e within
// 1e-9, tests/test_gpu_te_solver.py).  k_cooling, whose cooling lists feed the k-packet selection, keeps te_col_exc.
struct TeExcT {
  double inv_kT, A1, A2, A3;
};
DEVFN TeExcT te_exc_t(float T_e, float nne) {
  TeExcT f;
  f.inv_kT = 1. / (ARTIS_KB * T_e);
  f.A1 = ARTIS_C_0 * nne * sqrtf(T_e) * 14.51039491;
  f.A2 = nne * 8.629e-6 * 0.01 / sqrtf(T_e);
  f.A3 = nne * 8.629e-6 / sqrtf(T_e);
  return f;
}
DEVFN double te_col_exc_fast(const TeExcItem &it, const TeExcT &f, double inv_lsw) {
  const double coll_strength = it.coll_str;
  const double eoverkt = it.epsilon_trans * f.inv_kT;
  const bool allowed = coll_strength < 0 && !it.forbidden;
  const double ex = exp(allowed ? eoverkt : -eoverkt);
  const double lg = (allowed && eoverkt <= MA_GAUNT_NOLOG) ? log(eoverkt) : 0.;  // (Gamma = 0.2 above: physics.h)
  double C;
  if (allowed) {
    const double test = eoverkt > MA_GAUNT_NOLOG ? -1. : 0.276 * ex * (-0.5772156649 - lg);
    const double Gamma = 0.2 > test ? 0.2 : test;
    C = f.A1 * it.osc_f * it.P2 * eoverkt / ex * Gamma;
  } else if (coll_strength < 0) {
    C = f.A2 * ex * (double)it.upper_sw;
  } else {
    C = f.A3 * coll_strength * ex * inv_lsw;
  }
  return C;
}
// kpkt.cc:41-67 get_cooling_ion_coll_exc for one ion: its own serial sum over levels and up-transitions.  exact: the
// reference's expression term for term (te_col_exc, as k_cooling) -- the stored evaluation, whose totalcooling and
// cooling_contrib_ion the next transport's k-packet ion selection reads; the Brent iterations take te_col_exc_fast.
DEVNI double te_coll_exc_ion(const Ctx &K, const TeDev &D, const TeState &s, int ui, float T_e, float nne, bool exact) {
  const int e = K.T.ion_element[ui];
  const int ul0 = K.T.ion_uniqueleveloffset[ui];
  double C_exc = 0.;
  const int nlevels = K.T.ion_nlevels[ui];
  const TeExcT f = te_exc_t(T_e, nne);
  for (int level = 0; level < nlevels; level++) {
    const int ul = ul0 + level;
    const int nuptrans = K.T.level_nuptrans[ul];
    if (nuptrans == 0) continue;
    const double nnlevel = te_levelpop(K, D, s, e, ui, level);
    const double statweight = K.T.level_stat_weight[ul];
    const double inv_lsw = 1. / statweight;
    const TeExcItem *it = K.T.exc_items + K.T.level_uptrans_offset[ul];
    if (exact) {
      for (int ii = 0; ii < nuptrans; ii++) {
        const TeExcItem x = it[ii];
        C_exc += nnlevel * te_col_exc(x, T_e, nne, statweight) * x.epsilon_trans;
      }
      continue;
    }
#pragma unroll 2
    for (int ii = 0; ii < nuptrans; ii++) {
      const TeExcItem x = it[ii];
      const double C = nnlevel * te_col_exc_fast(x, f, inv_lsw) * x.epsilon_trans;
      C_exc += C;
    }
  }
  return C_exc;
}
// kpkt.cc:84-165 calculate_cooling_rates.  The cell's G lanes (s.g lanes from s.lane0, all on the same control path)
// split the per-ion collisional-excitation sums -- independent sums in the reference, each kept in its order -- and
// exchange them by lane shuffles; every lane then combines the ions in the reference's order.
DEVNI void te_cooling_rates(const Ctx &K, const TeDev &D, const TeState &s, TeRates *hc, bool store) {
  const float nne = D.nne[s.mgi];
  const float T_e = s.Te;
  const int ni = K.T.nions_total;
  double C_total = 0., C_ff_all = 0., C_fb_all = 0., C_exc_all = 0., C_ionization_all = 0.;
  // (T_e-only factors of the per-target terms, evaluated once: the same values the per-term calls compute)
  const LutT lt = lut_t(K, T_e);
  const double rsqrtT = pow((double)T_e, -0.5);
  for (int ub = 0; ub < ni; ub += s.g) {
    const int my_ui = ub + s.sub;
    double mine = 0.;
    if (my_ui < ni) mine = te_coll_exc_ion(K, D, s, my_ui, T_e, nne, store);
    for (int j = 0; j < s.g && ub + j < ni; j++) {
      const double C_exc = __shfl(mine, s.lane0 + j, 64);
      const int ui = ub + j;
      const int e = K.T.ion_element[ui];
      const int i = ui - K.T.elem_uniqueionoffset[e];
      const int nions = K.T.elem_nions[e];
      const int ul0 = K.T.ion_uniqueleveloffset[ui];
      double C_ion = 0.;
      const int nionisinglevels = K.T.ion_ionisinglevels[ui];
      const double nncurrention = te_ionstagepop(K, D, s, e, ui);
      const int ioncharge = K.T.ion_ionstage[ui] - 1;
      if (ioncharge > 0) {
        const double C_ff_ion = 1.426e-27 * sqrt((double)T_e) * pow((double)ioncharge, 2) * nncurrention * nne;
        C_ff_all += C_ff_ion;
        C_ion += C_ff_ion;
      }
      C_exc_all += C_exc;
      C_ion += C_exc;
      if (i < nions - 1) {
        const double nnupperion = te_ionstagepop(K, D, s, e, ui + 1);  // (the same for every target)
        for (int level = 0; level < nionisinglevels; level++) {
          const double epsilon_current = K.T.level_epsilon[ul0 + level];
          const double nnlevel = te_levelpop(K, D, s, e, ui, level);
          const int nt = get_nphixstargets(K, e, i, level);
          for (int t = 0; t < nt; t++) {
            const int upper = get_phixsupperlevel(K, e, i, level, t);
            const double epsilon_trans = epsilon(K, e, i + 1, upper) - epsilon_current;
            const double C =
                nnlevel * col_ionization_ratecoeff_r(K, T_e, nne, e, i, level, t, epsilon_trans, rsqrtT) * epsilon_trans;
            C_ionization_all += C;
            C_ion += C;
          }
          for (int t = 0; t < nt; t++) {
            const double C = lut_interp_at(K, K.T.bfcooling_coeff, e, i, level, t, T_e, lt) * nnupperion * nne;
            C_fb_all += C;
            C_ion += C;
          }
        }
      }
      C_total += C_ion;
      if (store) D.ccion[(int64_t)s.mgi * ni + ui] = C_ion;
    }
  }
  if (store) D.totcool[s.mgi] = C_total;
  if (hc) {
    hc->cooling_collisional = C_exc_all + C_ionization_all;
    hc->cooling_fb = C_fb_all;
    hc->cooling_ff = C_ff_all;
  }
}
// thermalbalance.cc:189-216 get_heating_ion_coll_deexc (DIRECT_COL_HEAT)
DEVNI double te_heating_ion_coll_deexc(const Ctx &K, const TeDev &D, const TeState &s, int ui, float T_e, float nne) {
  const int e = K.T.ion_element[ui];
  const int ul0 = K.T.ion_uniqueleveloffset[ui];
  double C_deexc = 0.;
  for (int level = 0; level < K.T.ion_nlevels[ui]; level++) {
    const int ul = ul0 + level;
    const int nd = K.T.level_ndowntrans[ul];
    if (nd == 0) continue;
    const double nnlevel = te_levelpop(K, D, s, e, ui, level);
    const double epsilon_level = K.T.level_epsilon[ul];
    const double statweight = K.T.level_stat_weight[ul];
    for (int k = 0; k < nd; k++) {
      const int li = K.T.downtrans_lineindex[K.T.level_downtrans_offset[ul] + k];
      const int lower = K.T.line_lower[li];
      const double epsilon_trans = epsilon_level - K.T.level_epsilon[ul0 + lower];
      C_deexc += nnlevel *
                 col_deexcitation_ratecoeff(K, T_e, nne, epsilon_trans, li, K.T.level_stat_weight[ul0 + lower], statweight) *
                 epsilon_trans;
    }
  }
  return C_deexc;
}
// thermalbalance.cc:218-346; the bf-heating sum over hb_ul (every element's ionising levels of its non-top ions)
DEVNI void te_heating_rates(const Ctx &K, const TeDev &D, const TeState &s, TeRates *hc) {
  double bfheating = 0.;
  const int64_t kk = D.hbk ? D.hbk[s.k] : s.k;
  const int64_t stride = D.hbk ? D.hbstride : D.ncells;
  for (int j = 0; j < D.nhb; j++) {
    const int ul = D.hb_ul[j];
    const int ui = K.T.level_ui[ul];
    const int e = K.T.ion_element[ui];
    const double nnlevel = te_levelpop(K, D, s, e, ui, ul - K.T.ion_uniqueleveloffset[ui]);
    bfheating += nnlevel * D.hbc[(int64_t)j * stride + kk];
  }
  if (D.direct_col_heat) {
    // the ions' sums added in unique-ion order (the bf sum is separate, so the reference's per-element interleaving
    // is immaterial); the cell's lanes split the ions as in te_cooling_rates
    double C_deexc = 0.;
    const int ni = K.T.nions_total;
    for (int ub = 0; ub < ni; ub += s.g) {
      const int my_ui = ub + s.sub;
      double mine = 0.;
      if (my_ui < ni) mine = te_heating_ion_coll_deexc(K, D, s, my_ui, s.Te, D.nne[s.mgi]);
      for (int j = 0; j < s.g && ub + j < ni; j++) C_deexc += __shfl(mine, s.lane0 + j, 64);
    }
    hc->heating_collisional = C_deexc;
  } else {
    hc->heating_collisional = D.colheat[s.mgi];
  }
  hc->heating_bf = bfheating;
  hc->heating_ff = D.ffheat[s.mgi];
}
// thermalbalance.cc:348-395
DEVNI double te_eqn(const Ctx &K, const TeDev &D, TeState &s, double T_e, TeRates *hc, int *fail) {
  s.Te = T_e;
  double nntot = 0.;
  if (D.mode == 1) {
    nntot = te_electron_densities(K, D, s);
  } else if (te_calculate_populations(K, D, s, &nntot) != 0) {
    *fail = 1;
    return NAN;
  }
  te_cooling_rates(K, D, s, hc, false);
  te_heating_rates(K, D, s, hc);
  hc->heating_dep = D.hdep ? D.hdep[s.mgi] : 0.;
  const double p = nntot * ARTIS_KB * T_e;
  const double volumetmin = D.vol[s.mgi];
  const double dV = 3 * volumetmin / pow(D.tmin, 3) * pow(D.t_current, 2);
  const double V = volumetmin * pow(D.t_current / D.tmin, 3);
  hc->cooling_adiabatic = p * dV / V;
  const double total_heating_rate = hc->heating_ff + hc->heating_bf + hc->heating_collisional + hc->heating_dep;
  const double total_coolingrate = hc->cooling_ff + hc->cooling_fb + hc->cooling_collisional + hc->cooling_adiabatic;
  return total_heating_rate - total_coolingrate;
}

// thermalbalance.cc:141-187 (NO_LUT_BFHEATING false) for the levels the heating sum visits; workitem = (j, cell)
__global__ void k_te_bfheat(Ctx K, TeDev D) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)D.nhb * D.ncells) return;
  const int j = (int)(idx / D.ncells);
  const int k = (int)(idx % D.ncells);
  const int mgi = D.mgi[k];
  const int ul = D.hb_ul[j];
  const int ui = K.T.level_ui[ul];
  const int e = K.T.ion_element[ui];
  const int i = ui - K.T.elem_uniqueionoffset[e];
  const int l = ul - K.T.ion_uniqueleveloffset[ui];
  double bfheatingcoeff = 0.;
  for (int t = 0; t < get_nphixstargets(K, e, i, l); t++) {
    const double T_R = D.TR[mgi];
    const double W = D.W[mgi];
    bfheatingcoeff += W * lut_interp(K, D.bfheat_lut, e, i, l, t, T_R);
  }
  const int g = K.T.level_closestgroundlevelcont[ul];
  if (g >= 0) bfheatingcoeff *= D.bfest[(int64_t)mgi * K.T.nelements * K.T.maxnions + g];
  D.hbc[(int64_t)j * D.ncells + k] = bfheatingcoeff;
}

// lanes per cell of k_te_solve: one per ion (the per-ion sums of te_cooling_rates / te_heating_rates), at most 64
static inline int te_lanes_per_cell(int nions) { return nions < 1 ? 1 : (nions > 64 ? 64 : nions); }
// one wave = floor(64 / g) cells, g lanes each (the last 64 mod g lanes idle); every lane of a group runs its cell's
// solution
__global__ __launch_bounds__(64, 4) void k_te_solve(const Ctx *__restrict__ Kp, const TeDev *__restrict__ Dp, int g) {
  // context and parameters by device pointer, copied into LDS: the solver's functions are not inlined (register
  // pressure), and a by-value kernel argument referenced from them would be copied to scratch; read through the
  // global copies every table pointer was a dependent global load in the per-line loops
  CTX_IN_LDS(Kp);
  __shared__ TeDev s_dev;
  static_assert(sizeof(TeDev) % 8 == 0, "TeDev is copied in 8-byte words");
  for (int i = threadIdx.x; i < (int)(sizeof(TeDev) / 8); i += blockDim.x)
    reinterpret_cast<uint64_t *>(&s_dev)[i] = reinterpret_cast<const uint64_t *>(Dp)[i];
  __syncthreads();
  const TeDev &D = s_dev;
  const int lane = threadIdx.x;
  if (lane / g >= 64 / g) return;  // (lanes past the last whole group)
  const int k = blockIdx.x * (64 / g) + lane / g;
  if (k >= D.ncells) return;  // whole groups leave together
  TeState s;
  s.k = k;
  s.g = g;
  s.sub = lane % g;
  s.lane0 = lane - s.sub;
  extern __shared__ double te_lds[];
  s.phi = te_lds + (lane / g) * K.T.nions_total;
  s.mgi = D.mgi[k];
  s.Te = D.Te[s.mgi];
  const int mgi = s.mgi;
  TeRates hc = {0., 0., 0., 0., 0., 0., 0., 0.};
  int iters = 0;
  int fail = 0;
  if (D.mode == 2) {
    te_cooling_rates(K, D, s, nullptr, true);
    return;
  }
  if (D.mode == 1) {
    // the nebular pass (update_grid.cc:819-838): call_T_e_finder alone, populations from the NLTE solution; the
    // last evaluation at the final T_e leaves n_e and the rates of that T_e
    const double T_min = D.T_min, T_max = D.T_max;
    const double T_e_old = s.Te;
    auto f = [&](double T) { return te_eqn(K, D, s, T, &hc, &fail); };
    double thermalmin = f(T_min);
    double thermalmax = f(T_max);
    if (!isfinite(thermalmin) || !isfinite(thermalmax)) thermalmax = thermalmin = -1;
    double T_e = 0.;
    iters = -1;
    if (thermalmin * thermalmax < 0) {
      TeBrent b;
      if (te_brent_set(b, f, T_min, T_max) != 0) fail = 1;
      for (int iternum = 0; iternum < 100 && !fail; iternum++) {
        if (te_brent_iterate(b, f) != 0) {
          fail = 1;
          break;
        }
        T_e = b.root;
        iters = iternum + 1;
        if (te_test_interval(b.x_lower, b.x_upper, 0, D.accuracy) != 1) break;
      }
    } else if (thermalmax < 0) {
      T_e = T_min;
    } else {
      T_e = T_max;
    }
    if (!fail) {
      if (T_e > 2 * T_e_old) {
        T_e = 2 * T_e_old;
        if (T_e > T_max) T_e = T_max;
      } else if (T_e < 0.5 * T_e_old) {
        T_e = 0.5 * T_e_old;
        if (T_e < T_min) T_e = T_min;
      }
      f(T_e);
    }
    if (fail) {
      atomicCAS(D.fail, 0, mgi + 1);
      return;
    }
    D.Te[mgi] = s.Te;
    if (D.rates) {
      double *r = D.rates + (int64_t)mgi * ARTIS_TE_NRATES;
      r[0] = hc.cooling_collisional;
      r[1] = hc.cooling_fb;
      r[2] = hc.cooling_ff;
      r[3] = hc.cooling_adiabatic;
      r[4] = hc.heating_collisional;
      r[5] = hc.heating_bf;
      r[6] = hc.heating_ff;
      r[7] = hc.heating_dep;
    }
    return;
  }
  if (te_use_lte_ratio(D, mgi)) {
    // update_grid.cc:1106-1125 (T_J from get_T_J_from_J is the caller's TJ)
    s.Te = D.TJ[mgi];
    te_precalculate_partfuncts(K, D, s);
    double nntot;
    if (te_calculate_populations(K, D, s, &nntot) != 0) fail = 1;
  } else {
    // solve_Te_nltepops without NLTE_POPS_ON (update_grid.cc:763-886): bf-heating coefficients (k_te_bfheat),
    // partition functions, call_T_e_finder (thermalbalance.cc:397-597), calculate_populations
    te_precalculate_partfuncts(K, D, s);
    const double T_min = D.T_min, T_max = D.T_max;
    const double T_e_old = s.Te;
    auto f = [&](double T) { return te_eqn(K, D, s, T, &hc, &fail); };
    double thermalmin = f(T_min);
    double thermalmax = f(T_max);
    if (!fail) {
      if (!isfinite(thermalmin) || !isfinite(thermalmax)) thermalmax = thermalmin = -1;
      double T_e = 0.;
      iters = -1;
      if (thermalmin * thermalmax < 0) {
        TeBrent b;
        if (te_brent_set(b, f, T_min, T_max) != 0) fail = 1;
        for (int iternum = 0; iternum < 100 && !fail; iternum++) {
          if (te_brent_iterate(b, f) != 0) {
            fail = 1;
            break;
          }
          T_e = b.root;
          iters = iternum + 1;
          if (te_test_interval(b.x_lower, b.x_upper, 0, D.accuracy) != 1) break;
        }
      } else if (thermalmax < 0) {
        T_e = T_min;
      } else {
        T_e = T_max;
      }
      if (!fail) {
        if (T_e > 2 * T_e_old) {
          T_e = 2 * T_e_old;
          if (T_e > T_max) T_e = T_max;
        } else if (T_e < 0.5 * T_e_old) {
          T_e = 0.5 * T_e_old;
          if (T_e < T_min) T_e = T_min;
        }
        s.Te = T_e;
        f(T_e);
        double nntot;
        if (!fail && te_calculate_populations(K, D, s, &nntot) != 0) fail = 1;
      }
    }
  }
  if (fail) {
    if (D.iters) D.iters[mgi] = -2;
    atomicCAS(D.fail, 0, mgi + 1);
    return;
  }
  te_cooling_rates(K, D, s, nullptr, true);
  D.Te[mgi] = s.Te;
  if (D.rates) {
    double *r = D.rates + (int64_t)mgi * ARTIS_TE_NRATES;
    r[0] = hc.cooling_collisional;
    r[1] = hc.cooling_fb;
    r[2] = hc.cooling_ff;
    r[3] = hc.cooling_adiabatic;
    r[4] = hc.heating_collisional;
    r[5] = hc.heating_bf;
    r[6] = hc.heating_ff;
    r[7] = hc.heating_dep;
  }
  if (D.iters) D.iters[mgi] = iters;
}

// ============================================================ update_grid_cell's estimator preparation
// (artis_gpu_prepare_temperatures; update_grid.cc:1041-1150, LTE options): one cell per workitem, in the reference's
// order.  Reads the previous T_R / W / T_J / T_e / n_e / populations, writes the normalised inputs of k_te_solve.
struct UgDev {
  const int32_t *mgi;
  int32_t ncells, nprocs, initial_iteration;
  double deltat, tratmid, T_min, T_max;
  const float *TR, *W, *TJ, *Te, *nne, *gp, *rho, *abund;
  const int16_t *thick;
  const double *vol, *J, *nuJ, *ff, *col, *gam, *bfh;
  const double *bfheat_lut;
  float *TR_out, *W_out, *TJ_out;
  double *ff_out, *col_out, *gam_out, *bfh_out, *renorm_out;
  int32_t *fail;  // first cell (mgi + 1) whose corrphotoionrenorm / bf-heating ratio is not finite (the reference's
                  // [fatal] aborts, update_grid.cc:911-918, 959-965)
};
// ltepop.cc:417-430 with the previous populations (NLTE_POPS_ON false)
DEVFN double ug_levelpop(const Ctx &K, const UgDev &U, int mgi, int e, int ui, int l) {
  const double raw = U.gp[(int64_t)mgi * K.T.nions_total + ui];
  const bool hasab = U.abund[(int64_t)mgi * K.T.nelements + e] > 0;
  const double nnground = raw < K.R.minpop ? (hasab ? K.R.minpop : 0.) : raw;
  double nn = nnground;
  if (l > 0) {
    const double T_exc = K.R.exc_te ? (double)U.Te[mgi] : (double)U.TJ[mgi];
    const double W = 1.;
    const int ul0 = K.T.ion_uniqueleveloffset[ui];
    nn = (nnground * W * (double)K.T.level_stat_weight[ul0 + l] / (double)K.T.level_stat_weight[ul0] *
          exp(-(K.T.level_epsilon[ul0 + l] - K.T.level_epsilon[ul0]) / ARTIS_KB / T_exc));
  }
  if (nn < K.R.minpop) nn = hasab ? K.R.minpop : 0.;
  return nn;
}
__global__ __launch_bounds__(256) void k_ug_prepare(const Ctx *__restrict__ Kp, const UgDev *__restrict__ Up) {
  const Ctx &K = *Kp;
  const UgDev &U = *Up;
  const int kk = blockIdx.x * blockDim.x + threadIdx.x;
  if (kk >= U.ncells) return;
  const int mgi = U.mgi[kk];
  const int nel = K.T.nelements, mx = K.T.maxnions;
  const int64_t row = (int64_t)mgi * nel * mx;
  const double deltaV = U.vol[mgi] * pow(U.tratmid, 3.);
  const double estimator_normfactor = 1 / deltaV / U.deltat / U.nprocs;
  const double estimator_normfactor_over4pi = ARTIS_ONEOVER4PI * estimator_normfactor;
  const double J = U.J[mgi] * estimator_normfactor_over4pi;
  float TR = U.TR[mgi], W = U.W[mgi], TJ = U.TJ[mgi];
  U.ff_out[mgi] = U.ff[mgi];
  U.col_out[mgi] = U.col[mgi];
  for (int q = 0; q < nel * mx; q++) {
    U.gam_out[row + q] = U.gam[row + q];
    U.bfh_out[row + q] = U.bfh[row + q];
  }
  if (U.initial_iteration || U.thick[mgi] == 1) {
    double T_J = pow(J * ARTIS_PI / ARTIS_STEBO, 1. / 4.);
    if (!isfinite(T_J))
      T_J = U.TR[mgi];
    else if (T_J > U.T_max)
      T_J = U.T_max;
    else if (T_J < U.T_min)
      T_J = U.T_min;
    TR = T_J;
    TJ = T_J;
    W = 1;
    for (int q = 0; q < nel * mx; q++) U.renorm_out[row + q] = 1.;
  } else {
    const double nuJ = U.nuJ[mgi] * estimator_normfactor_over4pi;
    U.ff_out[mgi] = U.ff[mgi] * estimator_normfactor;
    U.col_out[mgi] = U.col[mgi] * estimator_normfactor;
    const double W_old = U.W[mgi], TR_old = U.TR[mgi];
    for (int e = 0; e < nel; e++)
      for (int i = 0; i < K.T.elem_nions[e] - 1; i++) {
        const int64_t ix = row + e * mx + i;
        const double g = U.gam[ix] * (estimator_normfactor / ARTIS_H);
        U.renorm_out[ix] = g / (W_old * lut_interp(K, K.T.corrphotoioncoeff, e, i, 0, 0, TR_old));
        if (!isfinite(U.renorm_out[ix])) atomicCAS(U.fail, 0, mgi + 1);
      }
    const float T_e = U.Te[mgi];
    const float nne = U.nne[mgi];
    for (int e = 0; e < nel; e++)
      for (int i = 0; i < K.T.elem_nions[e] - 1; i++) {
        const int64_t ix = row + e * mx + i;
        const int ui = uion(K, e, i);
        double Gamma = 0., Col_ion = 0.;
        for (int level = 0; level < K.T.ion_nlevels[ui]; level++) {
          const double nnlevel = ug_levelpop(K, U, mgi, e, ui, level);
          for (int t = 0; t < get_nphixstargets(K, e, i, level); t++) {
            const int upperlevel = get_phixsupperlevel(K, e, i, level, t);
            double gammacorr = W_old * lut_interp(K, K.T.corrphotoioncoeff, e, i, level, t, TR_old);
            const int gi = K.T.level_closestgroundlevelcont[ulev(K, e, i, level)];
            if (gi >= 0) gammacorr *= U.renorm_out[row + gi];
            Gamma += nnlevel * gammacorr;
            const double epsilon_trans = epsilon(K, e, i + 1, upperlevel) - epsilon(K, e, i, level);
            Col_ion += nnlevel * col_ionization_ratecoeff(K, T_e, nne, e, i, level, t, epsilon_trans);
          }
        }
        Gamma += Col_ion;
        const double gpraw = U.gp[(int64_t)mgi * K.T.nions_total + ui];
        const double gpop = gpraw < K.R.minpop ? (U.abund[(int64_t)mgi * nel + e] > 0 ? K.R.minpop : 0.) : gpraw;
        Gamma /= gpop;  // get_groundlevelpop
        U.gam_out[ix] = Gamma;
        const double b = U.bfh[ix] * estimator_normfactor;
        const double ana = W_old * lut_interp(K, U.bfheat_lut, e, i, 0, 0, TR_old);
        U.bfh_out[ix] = b / ana;
        if (!isfinite(U.bfh_out[ix])) atomicCAS(U.fail, 0, mgi + 1);
      }
    const double nubar = nuJ / J;
    if (isfinite(nubar) && nubar != 0.) {
      float T_J = pow(J * ARTIS_PI / ARTIS_STEBO, 1 / 4.);
      if (T_J > U.T_max)
        T_J = U.T_max;
      else if (T_J < U.T_min)
        T_J = U.T_min;
      TJ = T_J;
      float T_R = ARTIS_H * nubar / ARTIS_KB / 3.832229494;
      if (T_R > U.T_max)
        T_R = U.T_max;
      else if (T_R < U.T_min)
        T_R = U.T_min;
      TR = T_R;
      W = J * ARTIS_PI / ARTIS_STEBO / pow((double)T_R, 4.);
    }
  }
  U.TR_out[mgi] = TR;
  U.W_out[mgi] = W;
  U.TJ_out[mgi] = TJ;
}
