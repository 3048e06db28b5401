// model_synth.cc -- synthetic ARTIS model generator (see model_synth.h).
//
// Builds, in the reference's own data layout conventions:
//   * atomic data: Fe/Co/Ni, ion stages II-V, single-level top ion (artisoptions_classic.h:34), levels with
//     energies/g, E1 + forbidden lines sorted by descending nu (input.cc:747-1186), phixs tables in the v2
//     interpolated form (atomic.cc:87-155), continuum lists sorted by nu_edge (input.cc:1439-1652), cooling
//     list (kpkt.cc:339-426) and rate-coefficient LUTs (ratecoeff.cc:450-620) integrated here by composite
//     Gauss-Legendre instead of GSL qag (input generation; both oracle and engine read the same LUTs);
//   * a uniform cuboid grid (grid.cc:2028-2102) carrying a 3D model (map_3dmodeltogrid, grid.cc:988) or a 1D
//     shell model (map_1dmodeltogrid, grid.cc:910);
//   * per-timestep LTE cell state (Saha-Boltzmann with a bisection for n_e) and the k-packet cooling totals of
//     calculate_cooling_rates (kpkt.cc:84-165) -- the update_grid stand-in;
//   * the pure r-packet initial ensemble of SURVEY.md §8(d).
#include "model_synth.h"

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <numeric>
#include <random>
#include <vector>

#include "artis_constants.h"
#include "artis_io.h"

namespace {

struct Model {
  artis_synth_config cfg{};
  // ---- atomic
  int nelements = 0, maxnions = 0, nions_total = 0, nlevels_total = 0, nlines = 0, nbfcontinua = 0,
      nbfcontinua_ground = 0, ncoolingterms = 0;
  int nphixspoints = 100;
  double nphixsnuincrement = 0.1;
  double last_phixs_nuovernuedge = 0.;
  int tablesize = 100;
  double mintemp = 3500., maxtemp = 140000.;
  std::vector<int32_t> elem_anumber, elem_nions, elem_uniqueionoffset;
  std::vector<double> elem_mass_amu;
  std::vector<int32_t> ion_ionstage, ion_nlevels, ion_uniqueleveloffset, ion_ionisinglevels,
      ion_maxrecombininglevel, ion_coolingoffset, ion_ncoolingterms, ion_element;
  std::vector<double> ion_ionpot;
  std::vector<double> level_epsilon;
  std::vector<float> level_stat_weight;
  std::vector<int32_t> level_nuptrans, level_uptrans_offset, level_ndowntrans, level_downtrans_offset,
      level_nphixstargets, level_phixstargets_offset, level_cont_index, level_closestgroundlevelcont,
      level_phixstable;
  std::vector<int32_t> uptrans_lineindex, downtrans_lineindex, phixstarget_levelindex;
  std::vector<double> phixstarget_probability;
  std::vector<float> phixs_xs;
  std::vector<double> line_nu;
  std::vector<float> line_A, line_f, line_coll;
  std::vector<int32_t> line_elem, line_ion, line_upper, line_lower;
  std::vector<uint8_t> line_forbidden;
  std::vector<double> allcont_nu_edge, allcont_probability;
  std::vector<int32_t> allcont_element, allcont_ion, allcont_level, allcont_target, allcont_upperlevel,
      allcont_phixstable, allcont_groundindex;
  std::vector<double> groundcont_nu_edge;
  std::vector<int32_t> groundcont_element, groundcont_ion, groundcont_level, groundcont_target;
  std::vector<double> spontrecombcoeff, corrphotoioncoeff, bfcooling_coeff;
  std::vector<double> bfheating_coeff;  // ratecoeff.cc:583-599 (update_grid's thermal balance)
  std::vector<float> ion_alpha_sp;      // [nions_total * tablesize] ratecoeff.cc:967-990
  artis_te_tables te_tables;
  std::vector<int32_t> cool_type, cool_element, cool_ion, cool_level, cool_upper;
  artis_atomic_tables at{};

  // ---- grid
  int ngrid = 0, npts_model = 0;
  std::vector<double> cell_pos_min;
  std::vector<double> cell_wid;  // GRID_SPHERICAL1D: wid_init(cellindex) = (vout - v_inner) tmin (grid.cc:76-91)
  std::vector<int32_t> cell_mgi;
  std::vector<double> ts_start, ts_width, ts_mid;
  std::vector<double> mgi_rho_tmin;  // density at tmin
  std::vector<double> mgi_vel;       // representative velocity
  std::vector<float> mgi_X;          // [npts_model * nelements]
  std::vector<int32_t> mgi_tclass;
  std::vector<double> tclass_T;
  // model read from the reference's input files (artis_model_from_files) instead of the synthetic profile
  bool from_files = false;
  artis_input_params inp{};
  std::vector<double> mgi_ffegrp, mgi_ni56, mgi_rpos;  // model.txt X_Fegroup / X_Ni56; mean radial pos at tmin
  double kappagrey_norm = 1.;                           // (0.9 mfeg / mtot) + 0.1 of calculate_kappagrey
  double tmin = 0, tmax = 0, vmax = 0, rmax = 0;
  artis_geometry geom{};

  // ---- cell state
  std::vector<float> Te, TR, TJ, W, nne, nnetot, rho, kappagrey;
  std::vector<int16_t> thick;
  std::vector<float> elem_abundance, groundlevelpop, partfunct;
  std::vector<double> totalcooling, cooling_contrib_ion, corrphotoionrenorm;
  std::vector<float> ffegrp;
  artis_cell_state cs{};
  // ---- nebular options (cfg.nebular)
  std::vector<int32_t> ion_nlevels_nlte, ion_first_nlte;
  int total_nlte_levels = 0;
  std::vector<double> rf_nu_upper;
  std::vector<double> nlte_pops, nt_dep, nt_Y;
  std::vector<float> rf_TR, rf_W, bfrate_est, nt_prob, nt_ionen;

  // ---- decay stand-in (decay.cc nuclides + gammapkt.cc gamma_spectra)
  static constexpr int NNUC = 5;
  std::vector<double> gl_energy[NNUC], gl_prob[NNUC];
  std::vector<int32_t> gs_nlines, gs_offset;
  std::vector<double> gs_endecay, gs_energy, gs_prob;
  artis_gamma_spectra gs{};
  int current_nts = -1;
};

inline int uniqueion(const Model &m, int element, int ion) { return m.elem_uniqueionoffset[element] + ion; }
inline int uniquelevel(const Model &m, int element, int ion, int level) {
  return m.ion_uniqueleveloffset[uniqueion(m, element, ion)] + level;
}

// atomic.cc:87-155 (v2 interpolated tables), returned through a float exactly as the reference does
float phixs_xs_at(const Model &m, int table, double nu_edge, double nu) {
  const float *xs = &m.phixs_xs[(size_t)table * m.nphixspoints];
  float sigma_bf;
  const double ireal = (nu / nu_edge - 1.0) / m.nphixsnuincrement;
  const int i = (int)floor(ireal);
  if (i < 0) {
    sigma_bf = 0.0;
  } else if (i < m.nphixspoints - 1) {
    const double a = xs[i];
    const double b = xs[i + 1];
    const double fb = ireal - i;
    sigma_bf = ((1. - fb) * a) + (fb * b);
  } else {
    const double nu_max_phixs = nu_edge * m.last_phixs_nuovernuedge;
    sigma_bf = xs[m.nphixspoints - 1] * pow(nu_max_phixs / nu, 3);
  }
  return sigma_bf;
}

// Composite Gauss-Legendre (8 points) over each phixs table interval of [nu_edge, nu_edge * last].
template <typename F>
double integrate_phixs_range(const Model &m, double nu_edge, F f) {
  static const double x8[8] = {-0.9602898564975363, -0.7966664774136267, -0.5255324099163290, -0.1834346424956498,
                               0.1834346424956498,  0.5255324099163290,  0.7966664774136267,  0.9602898564975363};
  static const double w8[8] = {0.1012285362903763, 0.2223810344533745, 0.3137066458778873, 0.3626837833783620,
                               0.3626837833783620, 0.3137066458778873, 0.2223810344533745, 0.1012285362903763};
  double sum = 0.;
  const int npieces = m.nphixspoints - 1;
  const double dnu = nu_edge * m.nphixsnuincrement;
  for (int p = 0; p < npieces; p++) {
    const double a = nu_edge + p * dnu;
    const double b = a + dnu;
    const double half = 0.5 * (b - a), mid = 0.5 * (a + b);
    for (int k = 0; k < 8; k++) sum += w8[k] * half * f(mid + half * x8[k]);
  }
  return sum;
}

double calculate_sahafact(const Model &m, int element, int ion, int level, int upperionlevel, double T,
                          double E_threshold) {
  // ltepop.cc:539-556
  const double g_lower = m.level_stat_weight[uniquelevel(m, element, ion, level)];
  const double g_upper = m.level_stat_weight[uniquelevel(m, element, ion + 1, upperionlevel)];
  return ARTIS_SAHACONST * g_lower / g_upper * pow(T, -1.5) * exp(E_threshold / ARTIS_KB / T);
}

double minpop_of(const Model &m) { return m.cfg.minpop > 0. ? m.cfg.minpop : (m.cfg.nebular ? 1e-40 : ARTIS_MINPOP); }

// deterministic uniform in [0, 1) from (a, b, salt) (splitmix64): the nebular stand-ins do not depend on the
// order cells are visited in
double hash_u01(uint64_t a, uint64_t b, uint64_t salt) {
  uint64_t z = a * 0x9E3779B97F4A7C15ull ^ (b + 0x632BE59BD9B4E019ull) * 0xBF58476D1CE4E5B9ull ^ salt * 0x94D049BB133111EBull;
  z ^= z >> 30;
  z *= 0xBF58476D1CE4E5B9ull;
  z ^= z >> 27;
  z *= 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (double)(z >> 11) * (1.0 / 9007199254740992.0);
}

// input.cc:1711-1746 (NLTE level bookkeeping, LEVEL_IS_NLTE contiguous from the ground state) and
// radfield.cc:131-188 setup_bin_boundaries (equal frequency bins + the top super bin)
void setup_nebular_atomic(Model &m) {
  artis_atomic_tables &a = m.at;
  if (!m.cfg.nebular) return;
  const int ni = m.nions_total;
  m.ion_nlevels_nlte.assign(ni, 0);
  m.ion_first_nlte.assign(ni, 0);
  m.total_nlte_levels = 0;
  for (int ui = 0; ui < ni; ui++) {
    m.ion_first_nlte[ui] = m.total_nlte_levels;
    const int nlevels = m.ion_nlevels[ui];
    const int n = std::max(0, std::min(nlevels - 1, m.cfg.nlte_level_max));
    m.ion_nlevels_nlte[ui] = n;
    m.total_nlte_levels += n + ((nlevels > n + 1) ? 1 : 0);
  }
  a.ion_nlevels_nlte = m.ion_nlevels_nlte.data();
  a.ion_first_nlte = m.ion_first_nlte.data();
  a.total_nlte_levels = m.total_nlte_levels;
  const int nb = m.cfg.radfield_nbins > 1 ? m.cfg.radfield_nbins : 256;
  const double nu_lower_first_initial = ARTIS_CLIGHT / (40000e-8);
  const double nu_upper_last_initial = ARTIS_CLIGHT / (1085e-8);
  const double nu_upper_superbin = ARTIS_CLIGHT / (10e-8);
  const double delta_nu = (nu_upper_last_initial - nu_lower_first_initial) / (nb - 1);
  m.rf_nu_upper.assign(nb, 0.);
  for (int b = 0; b < nb - 1; b++) m.rf_nu_upper[b] = nu_lower_first_initial + (b + 1) * delta_nu;
  m.rf_nu_upper[nb - 1] = nu_upper_superbin;
  a.radfield_nbins = nb;
  a.radfield_nu_upper = m.rf_nu_upper.data();
  a.radfield_nu_lower_first = nu_lower_first_initial;
}

int get_nphixstargets(const Model &m, int element, int ion, int level) {
  const int ui = uniqueion(m, element, ion);
  if (ion < m.elem_nions[element] - 1 && level < m.ion_ionisinglevels[ui])
    return m.level_nphixstargets[uniquelevel(m, element, ion, level)];
  return 0;
}

void build_atomic(Model &m, std::mt19937_64 &rng) {
  std::uniform_real_distribution<double> U(0., 1.);
  const int Zs[3] = {26, 27, 28};
  const double masses[3] = {55.845, 58.933, 58.693};
  // ionisation potentials [eV] of stages I..V
  const double ip0[3][5] = {{7.902, 16.199, 30.651, 54.91, 75.0},
                            {7.881, 17.084, 33.50, 51.27, 79.5},
                            {7.640, 18.169, 35.19, 54.92, 76.06}};
  const double ipscale = (m.cfg.ionpot_scale > 0.) ? m.cfg.ionpot_scale : 1.;
  double ionpots[3][5];
  for (int e = 0; e < 3; e++)
    for (int j = 0; j < 5; j++) ionpots[e][j] = ip0[e][j] * ipscale;
  m.nelements = 3;
  m.maxnions = 4;
  const int nlev = m.cfg.nlevels_per_ion;
  for (int e = 0; e < m.nelements; e++) {
    m.elem_anumber.push_back(Zs[e]);
    m.elem_nions.push_back(4);
    m.elem_mass_amu.push_back(masses[e]);
    m.elem_uniqueionoffset.push_back(m.nions_total);
    double eps_ionground = ionpots[e][0] * ARTIS_EV;  // stage II ground relative to neutral ground
    for (int ion = 0; ion < 4; ion++) {
      const int ionstage = ion + 2;
      const bool top = (ion == 3);
      const int nl = top ? 1 : nlev;
      m.ion_element.push_back(e);
      m.ion_ionstage.push_back(ionstage);
      m.ion_nlevels.push_back(nl);
      m.ion_uniqueleveloffset.push_back(m.nlevels_total);
      m.ion_ionisinglevels.push_back(top ? 0 : std::min(m.cfg.n_ionising, nl));
      m.ion_maxrecombininglevel.push_back(0);
      m.ion_ionpot.push_back(ionpots[e][ion + 1] * ARTIS_EV);
      // levels: epsilon relative to the neutral ground state (globals.h:86)
      const double emax = 0.72 * ionpots[e][ion + 1] * ARTIS_EV;
      std::vector<double> exc(nl, 0.);
      for (int l = 1; l < nl; l++) {
        const double x = (l + 0.3 * (U(rng) - 0.5)) / (double)nl;
        exc[l] = emax * pow(std::max(x, 1e-4), 1.35);
      }
      std::sort(exc.begin(), exc.end());
      for (int l = 0; l < nl; l++) {
        m.level_epsilon.push_back(eps_ionground + exc[l]);
        const int gchoices[6] = {2, 4, 6, 8, 10, 12};
        m.level_stat_weight.push_back((float)gchoices[(int)(U(rng) * 6) % 6]);
      }
      m.nlevels_total += nl;
      eps_ionground += ionpots[e][ion + 1] * ARTIS_EV;
    }
    m.nions_total += 4;
  }

  // ---- lines (E1 permitted + forbidden) between levels of the non-top ions
  struct L {
    double nu;
    float A, f, coll;
    int e, ion, up, lo;
    bool forb;
  };
  std::vector<L> lines;
  // connectivity: each level connects down to its line_window nearest lower levels and to the lowest
  // n_resonance levels (resonance-like lines), like the sparse transition lists of real atomic data
  const int W = std::max(1, m.cfg.line_window);
  const int NR = std::max(0, m.cfg.n_resonance);
  // 8 pi^2 e^2 / (m_e c^3): A_ul = f_lu * g_l/g_u * coef * nu^2
  const double coef = 8. * ARTIS_PI * ARTIS_PI * ARTIS_QE * ARTIS_QE / (ARTIS_ME * pow(ARTIS_CLIGHT, 3));
  for (int e = 0; e < m.nelements; e++) {
    for (int ion = 0; ion < 4; ion++) {
      const int ui = uniqueion(m, e, ion);
      const int nl = m.ion_nlevels[ui];
      for (int up = 1; up < nl; up++) {
        for (int lo = 0; lo < up; lo++) {
          if (!(lo >= up - W || lo < NR)) continue;
          if ((int)lines.size() >= m.cfg.max_lines) continue;
          const double eps_l = m.level_epsilon[uniquelevel(m, e, ion, lo)];
          const double eps_u = m.level_epsilon[uniquelevel(m, e, ion, up)];
          const double nu = (eps_u - eps_l) / ARTIS_H;
          if (!(nu > 0.)) continue;
          const double gl = m.level_stat_weight[uniquelevel(m, e, ion, lo)];
          const double gu = m.level_stat_weight[uniquelevel(m, e, ion, up)];
          L l{};
          l.nu = nu;
          l.e = e;
          l.ion = ion;
          l.up = up;
          l.lo = lo;
          l.forb = U(rng) < 0.2;
          double f;
          if (l.forb) {
            f = pow(10., -8. + 3. * U(rng));
            l.coll = -2.f;
          } else {
            f = pow(10., -4. + 4. * U(rng));
            l.coll = (U(rng) < 0.7) ? -1.f : (float)pow(10., -1. + 2. * U(rng));
          }
          l.f = (float)f;
          l.A = (float)(f * gl / gu * coef * nu * nu);
          lines.push_back(l);
        }
      }
    }
  }
  // descending nu; ties broken by (element, ion, lower, upper) for determinism
  std::stable_sort(lines.begin(), lines.end(), [](const L &a, const L &b) { return a.nu > b.nu; });
  m.nlines = (int)lines.size();
  for (const L &l : lines) {
    m.line_nu.push_back(l.nu);
    m.line_A.push_back(l.A);
    m.line_f.push_back(l.f);
    m.line_coll.push_back(l.coll);
    m.line_elem.push_back(l.e);
    m.line_ion.push_back(l.ion);
    m.line_upper.push_back(l.up);
    m.line_lower.push_back(l.lo);
    m.line_forbidden.push_back(l.forb ? 1 : 0);
  }
  // up/down transition lists (by ascending line index)
  std::vector<std::vector<int>> up(m.nlevels_total), down(m.nlevels_total);
  for (int li = 0; li < m.nlines; li++) {
    up[uniquelevel(m, m.line_elem[li], m.line_ion[li], m.line_lower[li])].push_back(li);
    down[uniquelevel(m, m.line_elem[li], m.line_ion[li], m.line_upper[li])].push_back(li);
  }
  for (int lv = 0; lv < m.nlevels_total; lv++) {
    m.level_nuptrans.push_back((int)up[lv].size());
    m.level_uptrans_offset.push_back((int)m.uptrans_lineindex.size());
    for (int li : up[lv]) m.uptrans_lineindex.push_back(li);
    m.level_ndowntrans.push_back((int)down[lv].size());
    m.level_downtrans_offset.push_back((int)m.downtrans_lineindex.size());
    for (int li : down[lv]) m.downtrans_lineindex.push_back(li);
  }

  // ---- photoionisation targets and tables (phixsdata_v2 form)
  m.last_phixs_nuovernuedge = 1.0 + m.nphixsnuincrement * (m.nphixspoints - 1);  // input.cc:253
  m.level_nphixstargets.assign(m.nlevels_total, 0);
  m.level_phixstargets_offset.assign(m.nlevels_total, 0);
  m.level_phixstable.assign(m.nlevels_total, -1);
  m.level_cont_index.assign(m.nlevels_total, 0);
  m.level_closestgroundlevelcont.assign(m.nlevels_total, -1);
  int ntables = 0;
  for (int e = 0; e < m.nelements; e++) {
    for (int ion = 0; ion < 3; ion++) {
      const int ui = uniqueion(m, e, ion);
      const int uiup = uniqueion(m, e, ion + 1);
      for (int lvl = 0; lvl < m.ion_ionisinglevels[ui]; lvl++) {
        const int ul = uniquelevel(m, e, ion, lvl);
        const int ntargets = (lvl == 0 && m.ion_nlevels[uiup] >= 2) ? 2 : 1;
        m.level_nphixstargets[ul] = ntargets;
        m.level_phixstargets_offset[ul] = (int)m.phixstarget_levelindex.size();
        for (int t = 0; t < ntargets; t++) {
          m.phixstarget_levelindex.push_back(t);
          m.phixstarget_probability.push_back(ntargets == 1 ? 1.0 : (t == 0 ? 0.7 : 0.3));
          m.ion_maxrecombininglevel[uiup] = std::max(m.ion_maxrecombininglevel[uiup], t);  // input.cc:150
        }
        m.level_phixstable[ul] = ntables++;
        const double fscale = pow(10., -1. + 2. * U(rng));
        for (int i = 0; i < m.nphixspoints; i++) {
          const double x = 1.0 + i * m.nphixsnuincrement;
          m.phixs_xs.push_back((float)(1e-18 * fscale * pow(x, -3.)));
        }
      }
    }
  }
  // cont_index (input.cc:1153-1160)
  int cont_index = -1;
  for (int e = 0; e < m.nelements; e++)
    for (int ion = 0; ion < 4; ion++) {
      const int ui = uniqueion(m, e, ion);
      for (int lvl = 0; lvl < m.ion_ionisinglevels[ui]; lvl++) {
        m.level_cont_index[uniquelevel(m, e, ion, lvl)] = cont_index;
        cont_index -= get_nphixstargets(m, e, ion, lvl);
      }
    }
  m.nbfcontinua = -1 - cont_index;

  auto phixs_threshold = [&](int e, int ion, int lvl, int t) {
    const int ul = uniquelevel(m, e, ion, lvl);
    const int upper = m.phixstarget_levelindex[m.level_phixstargets_offset[ul] + t];
    return m.level_epsilon[uniquelevel(m, e, ion + 1, upper)] - m.level_epsilon[ul];  // atomic.cc:437-453
  };

  // ground continua (input.cc:1497-1523), nlevels_groundterm = 1
  struct GC {
    double nu_edge;
    int e, ion, lvl, t;
  };
  std::vector<GC> gcs;
  for (int e = 0; e < m.nelements; e++)
    for (int ion = 0; ion < 3; ion++)
      for (int t = 0; t < get_nphixstargets(m, e, ion, 0); t++)
        gcs.push_back({phixs_threshold(e, ion, 0, t) / ARTIS_H, e, ion, 0, t});
  std::stable_sort(gcs.begin(), gcs.end(), [](const GC &a, const GC &b) { return a.nu_edge < b.nu_edge; });
  m.nbfcontinua_ground = (int)gcs.size();
  for (const GC &g : gcs) {
    m.groundcont_nu_edge.push_back(g.nu_edge);
    m.groundcont_element.push_back(g.e);
    m.groundcont_ion.push_back(g.ion);
    m.groundcont_level.push_back(g.lvl);
    m.groundcont_target.push_back(g.t);
  }
  // search_groundphixslist (input.cc:1399-1437)
  auto search_ground = [&](double nu_edge, int *index_in_est) {
    if (nu_edge < m.groundcont_nu_edge[0]) {
      *index_in_est = -1;
      return -1;
    }
    int i;
    for (i = 1; i < m.nbfcontinua_ground; i++)
      if (nu_edge < m.groundcont_nu_edge[i]) break;
    int index;
    if (i == m.nbfcontinua_ground) {
      index = i - 1;
    } else {
      const double left = nu_edge - m.groundcont_nu_edge[i - 1];
      const double right = m.groundcont_nu_edge[i] - nu_edge;
      index = (left <= right) ? i - 1 : i;
    }
    *index_in_est = m.groundcont_element[index] * m.maxnions + m.groundcont_ion[index];
    return index;
  };
  // all continua (input.cc:1528-1570), then sorted by nu_edge
  struct AC {
    double nu_edge, prob;
    int e, ion, lvl, t, upper, table, gidx;
  };
  std::vector<AC> acs;
  for (int e = 0; e < m.nelements; e++)
    for (int ion = 0; ion < 3; ion++) {
      const int ui = uniqueion(m, e, ion);
      for (int lvl = 0; lvl < m.ion_ionisinglevels[ui]; lvl++) {
        const int ul = uniquelevel(m, e, ion, lvl);
        for (int t = 0; t < get_nphixstargets(m, e, ion, lvl); t++) {
          AC a{};
          a.nu_edge = phixs_threshold(e, ion, lvl, t) / ARTIS_H;
          a.prob = m.phixstarget_probability[m.level_phixstargets_offset[ul] + t];
          a.e = e;
          a.ion = ion;
          a.lvl = lvl;
          a.t = t;
          a.upper = m.phixstarget_levelindex[m.level_phixstargets_offset[ul] + t];
          a.table = m.level_phixstable[ul];
          int iest;
          a.gidx = search_ground(a.nu_edge, &iest);
          m.level_closestgroundlevelcont[ul] = iest;
          acs.push_back(a);
        }
      }
    }
  std::stable_sort(acs.begin(), acs.end(), [](const AC &a, const AC &b) { return a.nu_edge < b.nu_edge; });
  for (const AC &a : acs) {
    m.allcont_nu_edge.push_back(a.nu_edge);
    m.allcont_probability.push_back(a.prob);
    m.allcont_element.push_back(a.e);
    m.allcont_ion.push_back(a.ion);
    m.allcont_level.push_back(a.lvl);
    m.allcont_target.push_back(a.t);
    m.allcont_upperlevel.push_back(a.upper);
    m.allcont_phixstable.push_back(a.table);
    m.allcont_groundindex.push_back(a.gidx);
  }

  // ---- LUTs on the log-T grid (ratecoeff.cc:450-620), index get_bflutindex (sn3d.h:64)
  const double T_step_log = (log(m.maxtemp) - log(m.mintemp)) / (m.tablesize - 1.);
  m.spontrecombcoeff.assign((size_t)m.tablesize * m.nbfcontinua, 0.);
  m.corrphotoioncoeff.assign((size_t)m.tablesize * m.nbfcontinua, 0.);
  m.bfcooling_coeff.assign((size_t)m.tablesize * m.nbfcontinua, 0.);
  m.bfheating_coeff.assign((size_t)m.tablesize * m.nbfcontinua, 0.);
  struct Job {
    int e, ion, lvl, t;
  };
  std::vector<Job> jobs;
  for (int e = 0; e < m.nelements; e++)
    for (int ion = 0; ion < 3; ion++) {
      const int ui = uniqueion(m, e, ion);
      for (int lvl = 0; lvl < m.ion_ionisinglevels[ui]; lvl++)
        for (int t = 0; t < get_nphixstargets(m, e, ion, lvl); t++) jobs.push_back({e, ion, lvl, t});
    }
#pragma omp parallel for schedule(dynamic)
  for (int j = 0; j < (int)jobs.size(); j++) {
    const Job jb = jobs[j];
    const int ul = uniquelevel(m, jb.e, jb.ion, jb.lvl);
    const int upper = m.phixstarget_levelindex[m.level_phixstargets_offset[ul] + jb.t];
    const double prob = m.phixstarget_probability[m.level_phixstargets_offset[ul] + jb.t];
    const double E_threshold = phixs_threshold(jb.e, jb.ion, jb.lvl, jb.t);
    const double nu_threshold = E_threshold / ARTIS_H;
    const int table = m.level_phixstable[ul];
    const int contindex = -1 - m.level_cont_index[ul] + jb.t;
    for (int iter = 0; iter < m.tablesize; iter++) {
      const float T_e = (float)(m.mintemp * exp(iter * T_step_log));
      const double T = T_e;
      const double sfac = calculate_sahafact(m, jb.e, jb.ion, jb.lvl, upper, T_e, E_threshold);
      const double alpha_sp = integrate_phixs_range(m, nu_threshold, [&](double nu) {
        const float s = phixs_xs_at(m, table, nu_threshold, nu);
        return ARTIS_TWOOVERCLIGHTSQUARED * s * pow(nu, 2) * exp(-ARTIS_HOVERKB * nu / T);
      });
      const double gammacorr = integrate_phixs_range(m, nu_threshold, [&](double nu) {
        const float s = phixs_xs_at(m, table, nu_threshold, nu);
        const double dbb = ARTIS_TWOHOVERCLIGHTSQUARED * pow(nu, 3) / expm1(ARTIS_HOVERKB * nu / T);
        return s * ARTIS_ONEOVERH / nu * dbb * (1 - exp(-ARTIS_HOVERKB * nu / T));
      });
      const double bfcool = integrate_phixs_range(m, nu_threshold, [&](double nu) {
        const float s = phixs_xs_at(m, table, nu_threshold, nu);
        return s * (nu - nu_threshold) * ARTIS_TWOHOVERCLIGHTSQUARED * nu * nu * exp(-ARTIS_HOVERKB * nu / T);
      });
      const size_t idx = (size_t)iter * m.nbfcontinua + contindex;
      m.spontrecombcoeff[idx] = alpha_sp * ARTIS_FOURPI * sfac * prob;
      m.corrphotoioncoeff[idx] = gammacorr * ARTIS_FOURPI * prob;
      m.bfcooling_coeff[idx] = bfcool * ARTIS_FOURPI * sfac * prob;
      // approx_bfheating_integrand_gsl (ratecoeff.cc:325-343)
      const double bfheat = integrate_phixs_range(m, nu_threshold, [&](double nu) {
        const float s = phixs_xs_at(m, table, nu_threshold, nu);
        const double dbb = ARTIS_TWOHOVERCLIGHTSQUARED * pow(nu, 3) / expm1(ARTIS_HOVERKB * nu / T);
        return s * (1 - nu_threshold / nu) * dbb * (1 - exp(-ARTIS_HOVERKB * nu / T));
      });
      m.bfheating_coeff[idx] = bfheat * ARTIS_FOURPI * prob;
    }
  }
  // precalculate_ion_alpha_sp (ratecoeff.cc:967-990): per ion, the sum of get_spontrecombcoeff (ratecoeff.cc:686-710)
  // over its ionising levels and their targets at every table temperature; the top ion keeps calloc's zeros
  m.ion_alpha_sp.assign((size_t)m.nions_total * m.tablesize, 0.f);
  for (int iter = 0; iter < m.tablesize; iter++) {
    const float T_e = m.mintemp * exp(iter * T_step_log);
    for (int e = 0; e < m.nelements; e++)
      for (int ion = 0; ion < m.elem_nions[e] - 1; ion++) {
        const int ui = uniqueion(m, e, ion);
        double zeta = 0.;
        for (int lvl = 0; lvl < m.ion_ionisinglevels[ui]; lvl++)
          for (int t = 0; t < get_nphixstargets(m, e, ion, lvl); t++) {
            const int contindex = -1 - m.level_cont_index[uniquelevel(m, e, ion, lvl)] + t;
            const int lowerindex = floor(log(T_e / m.mintemp) / T_step_log);
            double a_sp;
            if (lowerindex < m.tablesize - 1) {
              const int upperindex = lowerindex + 1;
              const double T_lower = m.mintemp * exp(lowerindex * T_step_log);
              const double T_upper = m.mintemp * exp(upperindex * T_step_log);
              const double f_upper = m.spontrecombcoeff[(size_t)upperindex * m.nbfcontinua + contindex];
              const double f_lower = m.spontrecombcoeff[(size_t)lowerindex * m.nbfcontinua + contindex];
              a_sp = (f_lower + (f_upper - f_lower) / (T_upper - T_lower) * (T_e - T_lower));
            } else {
              a_sp = m.spontrecombcoeff[(size_t)(m.tablesize - 1) * m.nbfcontinua + contindex];
            }
            zeta += a_sp;
          }
        m.ion_alpha_sp[(size_t)ui * m.tablesize + iter] = zeta;
      }
  }
  m.te_tables.bfheating_coeff = m.bfheating_coeff.data();
  m.te_tables.ion_alpha_sp = m.ion_alpha_sp.data();

  // ---- cooling list (kpkt.cc:313-426)
  m.ion_coolingoffset.assign(m.nions_total, 0);
  m.ion_ncoolingterms.assign(m.nions_total, 0);
  for (int e = 0; e < m.nelements; e++) {
    const int nions = m.elem_nions[e];
    for (int ion = 0; ion < nions; ion++) {
      const int ui = uniqueion(m, e, ion);
      m.ion_coolingoffset[ui] = (int)m.cool_type.size();
      auto add = [&](int type, int lvl, int upper) {
        m.cool_type.push_back(type);
        m.cool_element.push_back(e);
        m.cool_ion.push_back(ion);
        m.cool_level.push_back(lvl);
        m.cool_upper.push_back(upper);
      };
      if (m.ion_ionstage[ui] - 1 > 0) add(ARTIS_COOLINGTYPE_FF, -99, -99);
      for (int lvl = 0; lvl < m.ion_nlevels[ui]; lvl++) {
        const int ul = uniquelevel(m, e, ion, lvl);
        if (m.level_nuptrans[ul] > 0) add(ARTIS_COOLINGTYPE_COLLEXC, lvl, -1);
        if (ion < nions - 1 && lvl < m.ion_ionisinglevels[ui]) {
          const int nt = get_nphixstargets(m, e, ion, lvl);
          for (int t = 0; t < nt; t++)
            add(ARTIS_COOLINGTYPE_COLLION, lvl, m.phixstarget_levelindex[m.level_phixstargets_offset[ul] + t]);
          for (int t = 0; t < nt; t++)
            add(ARTIS_COOLINGTYPE_FB, lvl, m.phixstarget_levelindex[m.level_phixstargets_offset[ul] + t]);
        }
      }
      m.ion_ncoolingterms[ui] = (int)m.cool_type.size() - m.ion_coolingoffset[ui];
    }
  }
  m.ncoolingterms = (int)m.cool_type.size();

  artis_atomic_tables &a = m.at;
  a.nelements = m.nelements;
  a.maxnions = m.maxnions;
  a.nions_total = m.nions_total;
  a.nlevels_total = m.nlevels_total;
  a.nlines = m.nlines;
  a.nbfcontinua = m.nbfcontinua;
  a.nbfcontinua_ground = m.nbfcontinua_ground;
  a.ncoolingterms = m.ncoolingterms;
  a.nphixspoints = m.nphixspoints;
  a.nphixsnuincrement = m.nphixsnuincrement;
  a.last_phixs_nuovernuedge = m.last_phixs_nuovernuedge;
  a.phixs_file_version = 2;
  a.tablesize = m.tablesize;
  a.mintemp = m.mintemp;
  a.maxtemp = m.maxtemp;
  a.elem_anumber = m.elem_anumber.data();
  a.elem_nions = m.elem_nions.data();
  a.elem_uniqueionoffset = m.elem_uniqueionoffset.data();
  a.ion_ionstage = m.ion_ionstage.data();
  a.ion_nlevels = m.ion_nlevels.data();
  a.ion_uniqueleveloffset = m.ion_uniqueleveloffset.data();
  a.ion_ionisinglevels = m.ion_ionisinglevels.data();
  a.ion_maxrecombininglevel = m.ion_maxrecombininglevel.data();
  a.ion_coolingoffset = m.ion_coolingoffset.data();
  a.ion_ncoolingterms = m.ion_ncoolingterms.data();
  a.ion_ionpot = m.ion_ionpot.data();
  a.level_epsilon = m.level_epsilon.data();
  a.level_stat_weight = m.level_stat_weight.data();
  a.level_nuptrans = m.level_nuptrans.data();
  a.level_uptrans_offset = m.level_uptrans_offset.data();
  a.level_ndowntrans = m.level_ndowntrans.data();
  a.level_downtrans_offset = m.level_downtrans_offset.data();
  a.level_nphixstargets = m.level_nphixstargets.data();
  a.level_phixstargets_offset = m.level_phixstargets_offset.data();
  a.level_cont_index = m.level_cont_index.data();
  a.level_closestgroundlevelcont = m.level_closestgroundlevelcont.data();
  a.level_phixstable = m.level_phixstable.data();
  a.uptrans_lineindex = m.uptrans_lineindex.data();
  a.downtrans_lineindex = m.downtrans_lineindex.data();
  a.phixstarget_levelindex = m.phixstarget_levelindex.data();
  a.phixstarget_probability = m.phixstarget_probability.data();
  a.phixs_xs = m.phixs_xs.data();
  a.line_nu = m.line_nu.data();
  a.line_einstein_A = m.line_A.data();
  a.line_osc_strength = m.line_f.data();
  a.line_coll_str = m.line_coll.data();
  a.line_elementindex = m.line_elem.data();
  a.line_ionindex = m.line_ion.data();
  a.line_upperlevelindex = m.line_upper.data();
  a.line_lowerlevelindex = m.line_lower.data();
  a.line_forbidden = m.line_forbidden.data();
  a.allcont_nu_edge = m.allcont_nu_edge.data();
  a.allcont_element = m.allcont_element.data();
  a.allcont_ion = m.allcont_ion.data();
  a.allcont_level = m.allcont_level.data();
  a.allcont_phixstargetindex = m.allcont_target.data();
  a.allcont_upperlevel = m.allcont_upperlevel.data();
  a.allcont_phixstable = m.allcont_phixstable.data();
  a.allcont_probability = m.allcont_probability.data();
  a.allcont_index_in_groundphixslist = m.allcont_groundindex.data();
  a.groundcont_nu_edge = m.groundcont_nu_edge.data();
  a.groundcont_element = m.groundcont_element.data();
  a.groundcont_ion = m.groundcont_ion.data();
  a.groundcont_level = m.groundcont_level.data();
  a.groundcont_phixstargetindex = m.groundcont_target.data();
  a.spontrecombcoeff = m.spontrecombcoeff.data();
  a.corrphotoioncoeff = m.corrphotoioncoeff.data();
  a.bfcooling_coeff = m.bfcooling_coeff.data();
  a.coolinglist_type = m.cool_type.data();
  a.coolinglist_element = m.cool_element.data();
  a.coolinglist_ion = m.cool_ion.data();
  a.coolinglist_level = m.cool_level.data();
  a.coolinglist_upperlevel = m.cool_upper.data();
}

void finish_geometry(Model &m);

// GRID_SPHERICAL1D: spherical1d_grid_setup (grid.cc:2104-2131) with the spherical branch of map_1dmodeltogrid
// (grid.cc:910-940): one propagation cell per shell, cellindex == mgi (npts_model for a shell without density),
// pos_min[0] = v_inner tmin, wid_init = (vout - v_inner) tmin
static bool spherical(const Model &m) { return m.geom.grid_type == ARTIS_GRID_SPHERICAL1D; }

static void spherical_grid(Model &m, const double *vout) {
  const int np = m.npts_model;
  m.ngrid = np;
  m.cell_pos_min.assign((size_t)np * 3, 0.);
  m.cell_wid.assign(np, 0.);
  m.cell_mgi.assign(np, np);
  for (int c = 0; c < np; c++) {
    const double v_inner = c > 0 ? vout[c - 1] : 0.;
    m.cell_pos_min[(size_t)c * 3] = v_inner * m.tmin;
    m.cell_wid[c] = (vout[c] - v_inner) * m.tmin;
    m.cell_mgi[c] = (vout[c] >= 0. && m.mgi_rho_tmin[c] > 0) ? c : np;
  }
  m.geom.grid_type = ARTIS_GRID_SPHERICAL1D;
}

// vol_init_gridcell (grid.cc:112-124) at tmin
static double cell_volume(const Model &m, int c) {
  if (spherical(m)) {
    const double r_in = m.cell_pos_min[(size_t)c * 3], r_out = r_in + m.cell_wid[c];
    return 4. / 3. * ARTIS_PI * (pow(r_out, 3) - pow(r_in, 3));
  }
  return pow(2 * m.geom.coordmax[0] / m.cfg.ngrid_1d, 3);
}

void build_grid(Model &m) {
  const artis_synth_config &c = m.cfg;
  m.tmin = c.tmin_days * ARTIS_DAY;
  m.tmax = c.tmax_days * ARTIS_DAY;
  m.vmax = c.vmax;
  m.rmax = m.vmax * m.tmin;
  const int n = c.ngrid_1d;
  m.ngrid = n * n * n;
  double coordmax[3] = {m.vmax * m.tmin, m.vmax * m.tmin, m.vmax * m.tmin};
  m.cell_pos_min.resize((size_t)m.ngrid * 3);
  for (int idx = 0; idx < m.ngrid; idx++) {
    const int nxyz[3] = {idx % n, (idx / n) % n, (idx / (n * n)) % n};
    for (int ax = 0; ax < 3; ax++)
      m.cell_pos_min[(size_t)idx * 3 + ax] = -coordmax[ax] + (2 * nxyz[ax] * coordmax[ax] / n);  // grid.cc:2083
  }
  const double wid = 2 * coordmax[0] / n;
  auto radialpos = [&](int idx) {
    double d[3];
    for (int ax = 0; ax < 3; ax++) d[ax] = m.cell_pos_min[(size_t)idx * 3 + ax] + 0.5 * wid;
    return sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
  };
  // exponential density profile normalised to the ejecta mass (at tmin)
  const double rho0 = c.mass_msun * ARTIS_MSUN / (8. * ARTIS_PI * pow(c.v_e, 3) * pow(m.tmin, 3));
  auto rho_at_v = [&](double v) { return v > m.vmax ? 0. : rho0 * exp(-v / c.v_e); };
  auto X_at_v = [&](double v, float X[3]) {
    const double xni = 0.6 * exp(-pow(v / 6e8, 2));
    X[2] = (float)xni;
    X[1] = 0.1f;
    X[0] = (float)(1. - xni - 0.1);
  };
  // temperature classes (quantised T(v), see model_synth.h)
  const int ntc = std::max(1, c.n_tclasses);
  m.tclass_T.resize(ntc);
  for (int k = 0; k < ntc; k++) {
    const double v = (k + 0.5) / ntc * m.vmax;
    m.tclass_T[k] = c.T0 * (1. + 0.5 * exp(-v / 5e8));
  }
  auto tclass_of_v = [&](double v) { return std::min(ntc - 1, std::max(0, (int)(v / m.vmax * ntc))); };

  m.cell_mgi.assign(m.ngrid, 0);
  if (c.nshells_1d > 0) {
    const int ns = c.nshells_1d;
    m.npts_model = ns;
    std::vector<double> vout(ns);
    for (int s = 0; s < ns; s++) vout[s] = (s + 1) * m.vmax / ns;
    m.mgi_rho_tmin.resize(ns);
    m.mgi_vel.resize(ns);
    m.mgi_X.resize((size_t)ns * 3);
    m.mgi_tclass.resize(ns);
    for (int s = 0; s < ns; s++) {
      const double vmid = (s + 0.5) * m.vmax / ns;
      m.mgi_vel[s] = vmid;
      m.mgi_rho_tmin[s] = rho_at_v(vmid);
      X_at_v(vmid, &m.mgi_X[(size_t)s * 3]);
      m.mgi_tclass[s] = tclass_of_v(vmid);
    }
    if (c.grid_spherical) {
      spherical_grid(m, vout.data());
      finish_geometry(m);
      return;
    }
    for (int idx = 0; idx < m.ngrid; idx++) {  // map_1dmodeltogrid (grid.cc:910-940)
      const double rpos = radialpos(idx);
      const double vcell = rpos / m.tmin;
      if (rpos < m.rmax) {
        int mgi = 0;
        for (int i = 0; i < ns - 1; i++)
          if (vout[mgi] < vcell) mgi = i + 1;
        m.cell_mgi[idx] = (m.mgi_rho_tmin[mgi] > 0) ? mgi : m.npts_model;
      } else {
        m.cell_mgi[idx] = m.npts_model;
      }
    }
  } else {
    m.npts_model = m.ngrid;  // map_3dmodeltogrid: mgi == cellindex
    m.mgi_rho_tmin.resize(m.ngrid);
    m.mgi_vel.resize(m.ngrid);
    m.mgi_X.resize((size_t)m.ngrid * 3);
    m.mgi_tclass.resize(m.ngrid);
    for (int idx = 0; idx < m.ngrid; idx++) {
      const double v = radialpos(idx) / m.tmin;
      m.mgi_vel[idx] = v;
      m.mgi_rho_tmin[idx] = rho_at_v(v);
      X_at_v(v, &m.mgi_X[(size_t)idx * 3]);
      m.mgi_tclass[idx] = tclass_of_v(v);
      m.cell_mgi[idx] = (m.mgi_rho_tmin[idx] > 0) ? idx : m.npts_model;
    }
  }

  finish_geometry(m);
}

// Grid from the reference's model.txt / abundances.txt: uniform_grid_setup (grid.cc:2028-2102) with
// map_1dmodeltogrid (grid.cc:910-940) or map_3dmodeltogrid (grid.cc:988-1005), densities scaled to tmin
// (grid.cc:1302, 1565), and the masses of calc_totmassradionuclides (grid.cc:1602-1655) for kappagrey.
int build_grid_from_model(Model &m, const artis_ejecta_model &em, const std::vector<float> &abund) {
  artis_synth_config &c = m.cfg;
  m.tmin = m.inp.tmin_days * ARTIS_DAY;
  m.tmax = m.inp.tmax_days * ARTIS_DAY;
  m.vmax = em.vmax;
  m.rmax = m.vmax * m.tmin;
  if (!(m.vmax > 0) || sqrt(3 * m.vmax * m.vmax) >= ARTIS_CLIGHT) return ARTIS_ERR_BAD_ARGUMENT;  // grid.cc:2035
  if (em.model_type == 3) c.ngrid_1d = em.ncoord_model[0];
  const int n = c.ngrid_1d;
  m.ngrid = n * n * n;
  const double coordmax[3] = {m.rmax, m.rmax, m.rmax};
  m.cell_pos_min.resize((size_t)m.ngrid * 3);
  for (int idx = 0; idx < m.ngrid; idx++) {
    const int nxyz[3] = {idx % n, (idx / n) % n, (idx / (n * n)) % n};
    for (int ax = 0; ax < 3; ax++)
      m.cell_pos_min[(size_t)idx * 3 + ax] = -coordmax[ax] + (2 * nxyz[ax] * coordmax[ax] / n);
  }
  const double wid = 2 * coordmax[0] / n;
  auto radialpos = [&](int idx) {  // get_cellradialpos: distance of the cell centre at tmin
    double d[3];
    for (int ax = 0; ax < 3; ax++) d[ax] = m.cell_pos_min[(size_t)idx * 3 + ax] + 0.5 * wid;
    return sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
  };
  const int np = em.npts_model;
  m.npts_model = np;
  m.mgi_rho_tmin.assign(np, 0.);
  m.mgi_vel.assign(np, 0.);
  m.mgi_X.assign((size_t)np * 3, 0.f);
  m.mgi_tclass.assign(np, 0);
  m.mgi_ffegrp.assign(np, 0.);
  m.mgi_ni56.assign(np, 0.);
  m.mgi_rpos.assign(np, 0.);
  const double tratio3 = pow(em.t_model / m.tmin, 3);
  for (int mgi = 0; mgi < np; mgi++) {
    m.mgi_rho_tmin[mgi] = em.rho_model[mgi] * tratio3;
    m.mgi_ffegrp[mgi] = em.ffegrp[mgi];
    m.mgi_ni56[mgi] = em.x_ni56[mgi];
    for (int e = 0; e < 3; e++) m.mgi_X[(size_t)mgi * 3 + e] = abund[(size_t)mgi * 3 + e];
  }
  std::vector<int> nassoc(np, 0);
  m.cell_mgi.assign(m.ngrid, np);
  if (c.grid_spherical && em.model_type == 1) {
    spherical_grid(m, em.vout);
    for (int mgi = 0; mgi < np; mgi++) nassoc[mgi] = (m.cell_mgi[mgi] == mgi) ? 1 : 0;
  }
  for (int idx = 0; idx < (spherical(m) ? 0 : m.ngrid); idx++) {
    const double rpos = radialpos(idx);
    int mgi = np;
    if (em.model_type == 1) {
      if (rpos < m.rmax) {
        const double vcell = rpos / m.tmin;
        mgi = 0;
        for (int i = 0; i < np - 1; i++)
          if (em.vout[mgi] < vcell) mgi = i + 1;
        if (!(em.vout[mgi] >= 0. && m.mgi_rho_tmin[mgi] > 0)) mgi = np;
      }
    } else {
      mgi = (m.mgi_rho_tmin[idx] > 0) ? idx : np;
    }
    m.cell_mgi[idx] = mgi;
    if (mgi < np) {
      m.mgi_rpos[mgi] += rpos;
      nassoc[mgi]++;
    }
  }
  for (int mgi = 0; mgi < np; mgi++) {
    if (nassoc[mgi] > 0) m.mgi_rpos[mgi] /= nassoc[mgi];
    // the cell-state stand-in's temperature class: velocity of the shell middle (1D) or the cell centre (3D)
    m.mgi_vel[mgi] = (em.model_type == 1) ? 0.5 * ((mgi > 0 ? em.vout[mgi - 1] : 0.) + em.vout[mgi])
                                          : radialpos(mgi) / m.tmin;
  }
  // calc_totmassradionuclides: mtot and mfeg over the model cells with rho > 0
  double mtot = 0., mfeg = 0.;
  for (int mgi = 0; mgi < np; mgi++) {
    if (m.mgi_rho_tmin[mgi] <= 0.) continue;
    double vol;
    if (em.model_type == 1) {
      const double v_inner = (mgi == 0) ? 0. : em.vout[mgi - 1];
      vol = (pow(em.vout[mgi], 3) - pow(v_inner, 3)) * 4 * ARTIS_PI * pow(m.tmin, 3) / 3.;
    } else {
      vol = pow((2 * m.vmax * m.tmin), 3.) / (n * n * n);
    }
    mtot += m.mgi_rho_tmin[mgi] * vol;
    mfeg += m.mgi_rho_tmin[mgi] * vol * m.mgi_ffegrp[mgi];
  }
  m.kappagrey_norm = (mtot > 0.) ? (0.9 * mfeg / mtot) + 0.1 : 1.;
  const int ntc = std::max(1, c.n_tclasses);
  m.tclass_T.resize(ntc);
  for (int k = 0; k < ntc; k++) {
    const double v = (k + 0.5) / ntc * m.vmax;
    m.tclass_T[k] = c.T0 * (1. + 0.5 * exp(-v / 5e8));
  }
  for (int mgi = 0; mgi < np; mgi++)
    m.mgi_tclass[mgi] = std::min(ntc - 1, std::max(0, (int)(m.mgi_vel[mgi] / m.vmax * ntc)));
  return 0;
}

// time grid and geometry record shared by both grid builders (input.cc:2236-2243)
void finish_geometry(Model &m) {
  const artis_synth_config &c = m.cfg;
  const int n = c.ngrid_1d;
  m.ts_start.resize(c.ntstep);
  m.ts_width.resize(c.ntstep);
  m.ts_mid.resize(c.ntstep);
  for (int i = 0; i < c.ntstep; i++) {
    const double dlogt = (log(m.tmax) - log(m.tmin)) / c.ntstep;
    m.ts_start[i] = m.tmin * exp(i * dlogt);
    m.ts_mid[i] = m.tmin * exp((i + 0.5) * dlogt);
    m.ts_width[i] = (m.tmin * exp((i + 1) * dlogt)) - m.ts_start[i];
  }
  artis_geometry &g = m.geom;
  g.ngrid = m.ngrid;
  g.npts_model = m.npts_model;
  g.cell_pos_min = m.cell_pos_min.data();
  g.cell_mgi = m.cell_mgi.data();
  if (spherical(m)) {  // spherical1d_grid_setup: ncoordgrid = {npts_model, 1, 1}, coordmax = {rmax, 0, 0}
    g.ncoordgrid[0] = m.ngrid;
    g.ncoordgrid[1] = g.ncoordgrid[2] = 1;
    g.modelcell_wid_init = m.cell_wid.data();
    g.coordmax[0] = m.rmax;
    g.coordmax[1] = g.coordmax[2] = 0.;
  } else {
    g.grid_type = ARTIS_GRID_UNIFORM;
    g.ncoordgrid[0] = g.ncoordgrid[1] = g.ncoordgrid[2] = n;
    g.modelcell_wid_init = nullptr;
    for (int ax = 0; ax < 3; ax++) g.coordmax[ax] = m.rmax;
  }
  g.tmin = m.tmin;
  g.tmax = m.tmax;
  g.rmax = m.rmax;
  g.vmax = m.vmax;
  g.ntstep = c.ntstep;
  g.ts_start = m.ts_start.data();
  g.ts_width = m.ts_width.data();
  g.ts_mid = m.ts_mid.data();
  g.nu_min_r = c.nu_min_r > 0. ? c.nu_min_r : (c.nebular ? 1e13 : ARTIS_NU_MIN_R);
  g.nu_max_r = c.nu_max_r > 0. ? c.nu_max_r : ARTIS_NU_MAX_R;
}

// ---- LTE cell state (update_grid stand-in) --------------------------------------------------------------

// macroatom.h:107-150 col_excitation_ratecoeff / nne  (linear in nne)
double col_exc_over_nne(const Model &m, float T_e, int li, double epsilon_trans, double gl, double gu) {
  const double coll_strength = m.line_coll[li];
  const double eoverkt = epsilon_trans / (ARTIS_KB * T_e);
  double C;
  if (coll_strength < 0) {
    if (!m.line_forbidden[li]) {
      const double g_bar = 0.2;
      const double exp_eoverkt = exp(eoverkt);
      const double test = 0.276 * exp_eoverkt * (-0.5772156649 - log(eoverkt));
      const double Gamma = g_bar > test ? g_bar : test;
      C = ARTIS_C_0 * sqrt(T_e) * 14.51039491 * m.line_f[li] * pow(ARTIS_H_IONPOT / epsilon_trans, 2) * eoverkt /
          exp_eoverkt * Gamma;
    } else {
      C = 8.629e-6 * 0.01 * exp(-eoverkt) * gu / sqrt(T_e);
    }
  } else {
    C = 8.629e-6 * coll_strength * exp(-eoverkt) / gl / sqrt(T_e);
  }
  return C;
}

// Fe-group fraction stand-in (the 56Ni-rich core of a W7-like model) and the grey opacity of opacity_case 4
// style kappagrey = GREY_OP (0.9 ffegrp + 0.1) (grid.cc:629); a cell is thick when its grey optical depth
// across one cell width exceeds thick_tau (input.txt cell_is_optically_thick).  rho: the density at time t (m.rho[mgi]
// holds it rounded to float).
static void cell_grey(Model &m, int nts, double t, int mgi, double rho) {
  m.thick[mgi] = 0;
  if (m.from_files) {
    // model.txt X_Fegroup; calculate_kappagrey opacity_case 4 (grid.cc:670-673); the grey-depth thick-cell
    // rule of update_grid_cell (update_grid.cc:1162-1197, 1209-1212)
    m.ffegrp[mgi] = (float)m.mgi_ffegrp[mgi];
    m.kappagrey[mgi] = (float)(((0.9 * m.mgi_ffegrp[mgi]) + 0.1) * ARTIS_GREY_OP / m.kappagrey_norm);
    const double tratmid = t / m.tmin;
    if (m.inp.opacity_case == 4) {
      double radial_pos = m.mgi_rpos[mgi] * tratmid;
      if (spherical(m)) {  // the volume-averaged mean radius of the shell (update_grid.cc:1164-1169)
        const double r_inner = m.cell_pos_min[(size_t)mgi * 3] * tratmid;
        const double r_outer = r_inner + m.cell_wid[mgi] * tratmid;
        radial_pos = 3. / 4 * (pow(r_outer, 4.) - pow(r_inner, 4.)) / (pow(r_outer, 3) - pow(r_inner, 3.));
      }
      const double grey_optical_depth = (double)m.kappagrey[mgi] * (double)m.rho[mgi] * (m.rmax * tratmid - radial_pos);
      if (grey_optical_depth > m.inp.cell_is_optically_thick && nts < m.inp.num_grey_timesteps) m.thick[mgi] = 1;
    } else {
      m.thick[mgi] = 1;
    }
  } else {
    const double v = m.mgi_vel[mgi];
    m.ffegrp[mgi] = (float)(0.2 + 0.6 * exp(-(v / 6e8) * (v / 6e8)));
    m.kappagrey[mgi] = (float)(0.1 * (0.9 * m.ffegrp[mgi] + 0.1));
    if (m.cfg.thick_tau > 0) {
      const double wid_t = (spherical(m) ? m.cell_wid[mgi] : 2 * m.geom.coordmax[0] / m.cfg.ngrid_1d) * t / m.tmin;
      if (m.kappagrey[mgi] * rho * wid_t > m.cfg.thick_tau) m.thick[mgi] = 1;
    }
  }
}

void compute_cellstate(Model &m, int nts) {
  const double t = m.ts_mid[nts];
  const int np = m.npts_model;
  const int ne = m.nelements, ni = m.nions_total;
  m.Te.assign(np, 0.f);
  m.TR.assign(np, 0.f);
  m.TJ.assign(np, 0.f);
  m.W.assign(np, 1.f);
  m.nne.assign(np, 0.f);
  m.nnetot.assign(np, 0.f);
  m.rho.assign(np, 0.f);
  m.kappagrey.assign(np, 0.f);
  m.thick.assign(np, 0);
  m.ffegrp.assign(np, 0.f);
  m.elem_abundance.assign((size_t)np * ne, 0.f);
  m.groundlevelpop.assign((size_t)np * ni, 0.f);
  m.partfunct.assign((size_t)np * ni, 1.f);
  m.totalcooling.assign(np, 0.);
  m.cooling_contrib_ion.assign((size_t)np * ni, 0.);
  m.corrphotoionrenorm.assign((size_t)np * ne * m.maxnions, 1.);
  if (m.cfg.nebular) {
    m.nlte_pops.assign((size_t)np * std::max(m.total_nlte_levels, 1), -1.);
    m.rf_TR.assign((size_t)np * m.at.radfield_nbins, 0.f);
    m.rf_W.assign((size_t)np * m.at.radfield_nbins, -1.f);
    m.bfrate_est.assign((size_t)np * std::max(m.nbfcontinua, 1), 0.f);
    m.nt_dep.assign(np, 0.);
    m.nt_Y.assign((size_t)np * ni, 0.);
    m.nt_prob.assign((size_t)np * ni * 3, 0.f);
    m.nt_ionen.assign((size_t)np * ni * 3, 0.f);
  }

  // per temperature class: partition functions, and per-level collisional-excitation cooling / nne
  const int ntc = (int)m.tclass_T.size();
  std::vector<double> U((size_t)ntc * ni), Sexc((size_t)ntc * m.nlevels_total, 0.);
#pragma omp parallel for schedule(dynamic)
  for (int k = 0; k < ntc; k++) {
    const float T = (float)m.tclass_T[k];
    for (int ui = 0; ui < ni; ui++) {
      const int off = m.ion_uniqueleveloffset[ui];
      double s = 0.;
      for (int l = 0; l < m.ion_nlevels[ui]; l++)
        s += m.level_stat_weight[off + l] * exp(-(m.level_epsilon[off + l] - m.level_epsilon[off]) / ARTIS_KB / T);
      U[(size_t)k * ni + ui] = s;
    }
    for (int ul = 0; ul < m.nlevels_total; ul++) {
      double s = 0.;
      const double eps = m.level_epsilon[ul];
      const double gl = m.level_stat_weight[ul];
      for (int j = 0; j < m.level_nuptrans[ul]; j++) {
        const int li = m.uptrans_lineindex[m.level_uptrans_offset[ul] + j];
        const int ui = m.elem_uniqueionoffset[m.line_elem[li]] + m.line_ion[li];
        const int uu = m.ion_uniqueleveloffset[ui] + m.line_upper[li];
        const double et = m.level_epsilon[uu] - eps;
        s += col_exc_over_nne(m, T, li, et, gl, m.level_stat_weight[uu]) * et;
      }
      Sexc[(size_t)k * m.nlevels_total + ul] = s;
    }
  }

  const double T_step_log = (log(m.maxtemp) - log(m.mintemp)) / (m.tablesize - 1.);
#pragma omp parallel for schedule(dynamic, 64)
  for (int mgi = 0; mgi < np; mgi++) {
    const double rho = m.mgi_rho_tmin[mgi] * pow(m.tmin / t, 3);
    if (!(rho > 0)) continue;
    const int k = m.mgi_tclass[mgi];
    const float T = (float)m.tclass_T[k];
    m.Te[mgi] = m.TR[mgi] = T;
    m.TJ[mgi] = (m.cfg.tj_scale > 0.) ? (float)(m.cfg.tj_scale * T) : T;
    m.W[mgi] = 1.f;
    m.rho[mgi] = (float)rho;
    double nntot_e[8], nnetot = 0.;
    for (int e = 0; e < ne; e++) {
      const float X = m.mgi_X[(size_t)mgi * 3 + e];
      m.elem_abundance[(size_t)mgi * ne + e] = X;
      nntot_e[e] = rho * X / (m.elem_mass_amu[e] * ARTIS_MH);
      nnetot += nntot_e[e] * m.elem_anumber[e];
    }
    // Saha ionisation balance; bisection in log n_e
    std::vector<double> frac((size_t)ni);
    auto ionfracs = [&](double ne_) {
      double nfree = 0.;
      for (int e = 0; e < ne; e++) {
        const int nions = m.elem_nions[e];
        const int u0 = m.elem_uniqueionoffset[e];
        double rel[8];
        rel[0] = 1.;
        double sum = 1.;
        for (int ion = 1; ion < nions; ion++) {
          const double chi = m.ion_ionpot[u0 + ion - 1];
          // n_{i}/n_{i-1} = U_i/U_{i-1} T^1.5 exp(-chi/kT) / (SAHACONST n_e)
          const double r = U[(size_t)k * ni + u0 + ion] / U[(size_t)k * ni + u0 + ion - 1] * pow(T, 1.5) *
                           exp(-chi / ARTIS_KB / T) / (ARTIS_SAHACONST * ne_);
          rel[ion] = rel[ion - 1] * r;
          if (rel[ion] > 1e250) rel[ion] = 1e250;
          sum += rel[ion];
        }
        for (int ion = 0; ion < nions; ion++) {
          frac[u0 + ion] = rel[ion] / sum;
          nfree += nntot_e[e] * frac[u0 + ion] * (m.ion_ionstage[u0 + ion] - 1);
        }
      }
      return nfree;
    };
    double lo = log(1e-6 * nnetot + 1e-30), hi = log(nnetot);
    for (int it = 0; it < 200; it++) {
      const double mid = 0.5 * (lo + hi);
      if (ionfracs(exp(mid)) > exp(mid))
        lo = mid;
      else
        hi = mid;
    }
    const double nne_sol = exp(0.5 * (lo + hi));
    ionfracs(nne_sol);
    m.nne[mgi] = (float)nne_sol;
    m.nnetot[mgi] = (float)nnetot;
    cell_grey(m, nts, t, mgi, rho);
    for (int e = 0; e < ne; e++) {
      const int u0 = m.elem_uniqueionoffset[e];
      for (int ion = 0; ion < m.elem_nions[e]; ion++) {
        const int ui = u0 + ion;
        const double Uion = U[(size_t)k * ni + ui];
        const double nion = nntot_e[e] * frac[ui];
        m.partfunct[(size_t)mgi * ni + ui] = (float)Uion;
        m.groundlevelpop[(size_t)mgi * ni + ui] =
            (float)(nion * m.level_stat_weight[m.ion_uniqueleveloffset[ui]] / Uion);
      }
    }
    // cooling totals (kpkt.cc:84-165) with the level populations of ltepop.cc:307-430 (MINPOP clamp; NLTE and
    // superlevel populations under the nebular options)
    const float nne = m.nne[mgi];
    const double minpop = minpop_of(m);
    auto groundpop = [&](int e, int ui) {
      const double nn = m.groundlevelpop[(size_t)mgi * ni + ui];
      if (nn < minpop) return m.elem_abundance[(size_t)mgi * ne + e] > 0 ? minpop : 0.;
      return nn;
    };
    const double T_exc = (m.cfg.excitation_te || m.cfg.nebular) ? m.Te[mgi] : m.TJ[mgi];
    auto lte_nominpop = [&](int e, int ui, int l) {
      const int off = m.ion_uniqueleveloffset[ui];
      const double ng = groundpop(e, ui);
      if (l == 0) return ng;
      return ng * 1. * m.level_stat_weight[off + l] / m.level_stat_weight[off] *
             exp(-(m.level_epsilon[off + l] - m.level_epsilon[off]) / ARTIS_KB / T_exc);
    };
    auto sl_boltzmann = [&](int ui, int l) {
      const int off = m.ion_uniqueleveloffset[ui];
      const int sl = m.ion_nlevels_nlte[ui] + 1;
      return (double)m.level_stat_weight[off + l] / m.level_stat_weight[off + sl] *
             exp(-(m.level_epsilon[off + l] - m.level_epsilon[off + sl]) / ARTIS_KB / T_exc);
    };
    if (m.cfg.nebular) {
      // NLTE population stand-in: LTE / rho times a factor in [0.5, 2); some ions without a solution (-1, the
      // "no NLTE information yet" marker of ltepop.cc:367); the superlevel from the LTE sum over its levels
      double *np_row = &m.nlte_pops[(size_t)mgi * m.total_nlte_levels];
      for (int ui = 0; ui < ni; ui++) {
        const int e = m.ion_element[ui];
        const int n = m.ion_nlevels_nlte[ui];
        const int f0 = m.ion_first_nlte[ui];
        const bool none = ((mgi + ui) % 7) == 3;
        for (int l = 1; l <= n; l++)
          np_row[f0 + l - 1] = none ? -1. : lte_nominpop(e, ui, l) / m.rho[mgi] * (0.5 + 1.5 * hash_u01(mgi, f0 + l, 11));
        if (m.ion_nlevels[ui] > n + 1) {
          double sum = 0., part = 0.;
          for (int l = n + 1; l < m.ion_nlevels[ui]; l++) {
            sum += lte_nominpop(e, ui, l);
            part += sl_boltzmann(ui, l);
          }
          np_row[f0 + n] = (((mgi + ui) % 5) == 1) ? -1. : sum / part / m.rho[mgi] * (0.5 + 1.5 * hash_u01(mgi, ui, 12));
        }
      }
    }
    auto levelpop = [&](int e, int ui, int l) {
      double nn = lte_nominpop(e, ui, l);
      if (l > 0 && m.cfg.nebular) {
        const double *np_row = &m.nlte_pops[(size_t)mgi * m.total_nlte_levels + m.ion_first_nlte[ui]];
        const int n = m.ion_nlevels_nlte[ui];
        const double v = (l <= n) ? np_row[l - 1] : np_row[n];
        if (!(v < -0.9)) return (l <= n) ? v * m.rho[mgi] : v * m.rho[mgi] * sl_boltzmann(ui, l);
      }
      if (nn < minpop) nn = m.elem_abundance[(size_t)mgi * ne + e] > 0 ? minpop : 0.;
      return nn;
    };
    auto ionstagepop = [&](int e, int ui) {
      return groundpop(e, ui) * m.partfunct[(size_t)mgi * ni + ui] /
             m.level_stat_weight[m.ion_uniqueleveloffset[ui]];
    };
    double C_total = 0.;
    for (int e = 0; e < ne; e++) {
      const int nions = m.elem_nions[e];
      for (int ion = 0; ion < nions; ion++) {
        const int ui = m.elem_uniqueionoffset[e] + ion;
        double C_ion = 0.;
        const double nncurrention = ionstagepop(e, ui);
        const int ioncharge = m.ion_ionstage[ui] - 1;
        if (ioncharge > 0) C_ion += 1.426e-27 * sqrt(T) * pow(ioncharge, 2) * nncurrention * nne;
        for (int l = 0; l < m.ion_nlevels[ui]; l++)
          C_ion += levelpop(e, ui, l) * nne * Sexc[(size_t)k * m.nlevels_total + m.ion_uniqueleveloffset[ui] + l];
        if (ion < nions - 1) {
          for (int l = 0; l < m.ion_ionisinglevels[ui]; l++) {
            const int ul = m.ion_uniqueleveloffset[ui] + l;
            const double nnlevel = levelpop(e, ui, l);
            const double epsilon_current = m.level_epsilon[ul];
            const int nt = get_nphixstargets(m, e, ion, l);
            for (int tg = 0; tg < nt; tg++) {
              const int upper = m.phixstarget_levelindex[m.level_phixstargets_offset[ul] + tg];
              const double eps_trans =
                  m.level_epsilon[m.ion_uniqueleveloffset[ui + 1] + upper] - epsilon_current;
              // macroatom.cc:745-776 col_ionization_ratecoeff
              const int ionstage = m.ion_ionstage[ui];
              const double g = (ionstage == 1) ? 0.1 : ((ionstage == 2) ? 0.2 : 0.3);
              const double fac1 = eps_trans / ARTIS_KB / T;
              const double sigma_bf = m.phixs_xs[(size_t)m.level_phixstable[ul] * m.nphixspoints] *
                                      m.phixstarget_probability[m.level_phixstargets_offset[ul] + tg];
              const double Ccol = nne * 1.55e13 * pow(T, -0.5) * g * sigma_bf * exp(-fac1) / fac1;
              C_ion += nnlevel * Ccol * eps_trans;
            }
            for (int tg = 0; tg < nt; tg++) {
              const double nnupperion = ionstagepop(e, ui + 1);
              // kpkt.cc:69-82 get_bfcoolingcoeff
              const int contindex = -1 - m.level_cont_index[ul] + tg;
              const int lowerindex = (int)floor(log(T / m.mintemp) / T_step_log);
              double bfc;
              if (lowerindex < m.tablesize - 1) {
                const int upperindex = lowerindex + 1;
                const double T_lower = m.mintemp * exp(lowerindex * T_step_log);
                const double T_upper = m.mintemp * exp(upperindex * T_step_log);
                const double f_upper = m.bfcooling_coeff[(size_t)upperindex * m.nbfcontinua + contindex];
                const double f_lower = m.bfcooling_coeff[(size_t)lowerindex * m.nbfcontinua + contindex];
                bfc = f_lower + (f_upper - f_lower) / (T_upper - T_lower) * (T - T_lower);
              } else {
                bfc = m.bfcooling_coeff[(size_t)(m.tablesize - 1) * m.nbfcontinua + contindex];
              }
              C_ion += bfc * nnupperion * nne;
            }
          }
        }
        C_total += C_ion;
        m.cooling_contrib_ion[(size_t)mgi * ni + ui] = C_ion;
      }
    }
    m.totalcooling[mgi] = C_total;
    if (m.cfg.nebular) {
      // binned radiation field fits within 5-10 % of the cell's T_R / W (radfield.cc:908-920), some bins without
      // a fit
      const int nb = m.at.radfield_nbins;
      for (int b = 0; b < nb; b++) {
        const size_t mb = (size_t)mgi * nb + b;
        m.rf_TR[mb] = (float)(m.TR[mgi] * (0.95 + 0.1 * hash_u01(mgi, b, 21)));
        m.rf_W[mb] = ((b % 13) == 5) ? -1.f : (float)(m.W[mgi] * (0.9 + 0.2 * hash_u01(mgi, b, 22)));
      }
      // normalised bf-rate estimators of a previous timestep: W * LUT(T_R) of the cell (ratecoeff.cc:1026-1041)
      // times a factor in [0.5, 1.5), some absent
      const int lowerindex = std::min((int)floor(log(m.TR[mgi] / m.mintemp) / T_step_log), m.tablesize - 2);
      const double fT = (m.TR[mgi] - m.mintemp * exp(lowerindex * T_step_log)) /
                        (m.mintemp * exp((lowerindex + 1) * T_step_log) - m.mintemp * exp(lowerindex * T_step_log));
      for (int i = 0; i < m.nbfcontinua; i++) {
        const int e = m.allcont_element[i], ion = m.allcont_ion[i], l = m.allcont_level[i], t = m.allcont_target[i];
        const int contindex = -1 - m.level_cont_index[uniquelevel(m, e, ion, l)] + t;
        const double lo = m.corrphotoioncoeff[(size_t)std::max(lowerindex, 0) * m.nbfcontinua + contindex];
        const double hi = m.corrphotoioncoeff[(size_t)(std::max(lowerindex, 0) + 1) * m.nbfcontinua + contindex];
        const double v = m.W[mgi] * (lo + (hi - lo) * std::max(0., fT)) * (0.5 + hash_u01(mgi, i, 23));
        m.bfrate_est[(size_t)mgi * m.nbfcontinua + i] = (i % 9 == 4) ? 0.f : ((i % 11 == 7) ? -1.f : (float)v);
      }
      // Spencer-Fano solution stand-in: ionisation rate coefficients, Auger-electron probabilities, and the
      // deposition rate density that makes the ionisation fraction of do_ntlepton 0.3 .. 0.8
      const int A = 2;
      double enrate_total = 0.;
      for (int e = 0; e < ne; e++) {
        const int nions = m.elem_nions[e];
        for (int ion = 0; ion < nions; ion++) {
          const int ui = m.elem_uniqueionoffset[e] + ion;
          m.nt_Y[(size_t)mgi * ni + ui] = (ion < nions - 1) ? pow(10., 1. + 3. * hash_u01(mgi, ui, 31)) : 0.;
          const double p0 = 0.7 + 0.2 * hash_u01(mgi, ui, 32), p1 = (1. - p0) * 0.7;
          const double q0 = 0.6 + 0.3 * hash_u01(mgi, ui, 33), q1 = (1. - q0) * 0.6;
          float *pr = &m.nt_prob[((size_t)mgi * ni + ui) * (A + 1)];
          float *pe = &m.nt_ionen[((size_t)mgi * ni + ui) * (A + 1)];
          pr[0] = (float)p0;
          pr[1] = (float)p1;
          pr[2] = (float)(1. - p0 - p1);
          pe[0] = (float)q0;
          pe[1] = (float)q1;
          pe[2] = (float)(1. - q0 - q1);
        }
        for (int lowerion = 0; lowerion < nions - 1; lowerion++) {
          const int ui = m.elem_uniqueionoffset[e] + lowerion;
          const double nnlowerion = groundpop(e, ui) * m.partfunct[(size_t)mgi * ni + ui] /
                                    m.level_stat_weight[m.ion_uniqueleveloffset[ui]];
          const int maxupper = std::min(lowerion + 1 + A, nions - 1);
          double enrate = 0.;
          for (int upperion = lowerion + 1; upperion <= maxupper; upperion++) {
            const float *pr = &m.nt_prob[((size_t)mgi * ni + ui) * (A + 1)];
            const int na = upperion - lowerion - 1;
            const double prob = (na < A) ? pr[na] : 1. - pr[0] - pr[1];
            enrate += nnlowerion * prob *
                      (m.level_epsilon[m.ion_uniqueleveloffset[ui + upperion - lowerion]] -
                       m.level_epsilon[m.ion_uniqueleveloffset[ui]]);
          }
          enrate_total += m.nt_Y[(size_t)mgi * ni + ui] * enrate;
        }
      }
      const double frac = 0.3 + 0.5 * hash_u01(mgi, 0, 34);
      m.nt_dep[mgi] = enrate_total > 0. ? enrate_total / frac : 1.;
    }
  }

  artis_cell_state &cs = m.cs;
  cs.Te = m.Te.data();
  cs.TR = m.TR.data();
  cs.TJ = m.TJ.data();
  cs.W = m.W.data();
  cs.nne = m.nne.data();
  cs.nnetot = m.nnetot.data();
  cs.rho = m.rho.data();
  cs.kappagrey = m.kappagrey.data();
  cs.thick = m.thick.data();
  cs.elem_abundance = m.elem_abundance.data();
  cs.groundlevelpop = m.groundlevelpop.data();
  cs.partfunct = m.partfunct.data();
  cs.totalcooling = m.totalcooling.data();
  cs.cooling_contrib_ion = m.cooling_contrib_ion.data();
  cs.corrphotoionrenorm = m.corrphotoionrenorm.data();
  cs.ffegrp = m.ffegrp.data();
  if (m.cfg.nebular) {
    cs.nlte_pops = m.nlte_pops.data();
    cs.radfield_bin_TR = m.rf_TR.data();
    cs.radfield_bin_W = m.rf_W.data();
    cs.bfrate_estimator = m.bfrate_est.data();
    cs.nt_deposition_rate_density = m.nt_dep.data();
    cs.nt_ionization_ratecoeff = m.nt_Y.data();
    cs.nt_prob_num_auger = m.nt_prob.data();
    cs.nt_ionenfrac_num_auger = m.nt_ionen.data();
  }
  m.current_nts = nts;
}


// ---------------------------------------------------------------------------------------- decay stand-in
// Five stand-in nuclides (decay.cc nuclides[]): mean life [d], particle energy per decay [MeV] and its decay
// type; the gamma energy per decay is the line-list sum (read_gamma_spectrum, gammapkt.cc:74-81) or, for the
// Fe52-like nuclide, set without a line list (gammapkt.cc:183-185).
struct NucDef {
  double meanlife_d, e_particle_mev, e_gamma_nolines_mev;
};
const NucDef kNuc[Model::NNUC] = {
    {6.075 / 0.69314718056, 0., 0.},        // 0 Ni56: EC
    {77.236 / 0.69314718056, 0.1158, 0.},   // 1 Co56: EC / beta+ (branch-weighted positron KE)
    {8.275 / 24. / 0.69314718056, 0., 0.86},// 2 Fe52-like: gamma energy, no line list
    {20., 0.3, 0.},                         // 3 beta- emitter
    {50., 5.0, 0.},                         // 4 alpha emitter
};
// decay paths (decay.cc decaypaths[]): chain of nuclides, final decay type, share of the decay energy
struct PathDef {
  int len, nuc[2], decaytype;
  double share;
};
const PathDef kPath[] = {
    {1, {0, -1}, ARTIS_DECAYTYPE_ELECTRONCAPTURE, 0.30},
    {2, {0, 1}, ARTIS_DECAYTYPE_ELECTRONCAPTURE, 0.30},
    {2, {0, 1}, ARTIS_DECAYTYPE_BETAPLUS, 0.10},
    {1, {2, -1}, ARTIS_DECAYTYPE_ELECTRONCAPTURE, 0.10},
    {1, {3, -1}, ARTIS_DECAYTYPE_BETAMINUS, 0.10},
    {1, {4, -1}, ARTIS_DECAYTYPE_ALPHA, 0.10},
};
constexpr int kNPath = sizeof(kPath) / sizeof(kPath[0]);

void rebuild_gamma_spectra(Model &m) {
  m.gs_nlines.assign(Model::NNUC, 0);
  m.gs_offset.assign(Model::NNUC, 0);
  m.gs_endecay.assign(Model::NNUC, 0.);
  m.gs_energy.clear();
  m.gs_prob.clear();
  for (int n = 0; n < Model::NNUC; n++) {
    m.gs_offset[n] = (int32_t)m.gs_energy.size();
    m.gs_nlines[n] = (int32_t)m.gl_energy[n].size();
    double eavg = 0.;
    for (size_t j = 0; j < m.gl_energy[n].size(); j++) {
      const double en = m.gl_energy[n][j] * ARTIS_MEV;
      m.gs_energy.push_back(en);
      m.gs_prob.push_back(m.gl_prob[n][j]);
      eavg += en * m.gl_prob[n][j];
    }
    m.gs_endecay[n] = m.gs_nlines[n] > 0 ? eavg : kNuc[n].e_gamma_nolines_mev * ARTIS_MEV;
  }
  m.gs.nnuclides = Model::NNUC;
  m.gs.nuc_nlines = m.gs_nlines.data();
  m.gs.nuc_line_offset = m.gs_offset.data();
  m.gs.nuc_endecay_gamma = m.gs_endecay.data();
  m.gs.line_energy = m.gs_energy.data();
  m.gs.line_probability = m.gs_prob.data();
}

}  // namespace

struct artis_model : Model {};

namespace {

// Every floating-point table the engine and the oracle read must be finite: a NaN here would propagate into both
// sides identically and hide (or fake) a parity mismatch.  Names the first offending array on stderr.
template <class V>
bool all_finite(const V &v, const char *name) {
  for (size_t k = 0; k < v.size(); k++)
    if (!std::isfinite((double)v[k])) {
      std::fprintf(stderr, "artis_model: %s[%zu] = %g is not finite\n", name, k, (double)v[k]);
      return false;
    }
  return true;
}

// the configuration's physical scalars: finite, and positive where the profile divides by or takes logs of them
bool config_is_sane(const artis_synth_config &c) {
  const double pos[] = {c.tmin_days, c.tmax_days, c.vmax, c.mass_msun, c.v_e, c.T0};
  const char *names[] = {"tmin_days", "tmax_days", "vmax", "mass_msun", "v_e", "T0"};
  for (int k = 0; k < 6; k++)
    if (!(std::isfinite(pos[k]) && pos[k] > 0)) {
      std::fprintf(stderr, "artis_model: config %s = %g must be finite and > 0\n", names[k], pos[k]);
      return false;
    }
  const double nonneg[] = {c.ionpot_scale, c.thick_tau, c.kpktdiffusion_timescale, c.tj_scale, c.minpop, c.nu_min_r,
                           c.nu_max_r};
  for (double v : nonneg)
    if (!(std::isfinite(v) && v >= 0)) {
      std::fprintf(stderr, "artis_model: a config scalar (%g) is negative or not finite\n", v);
      return false;
    }
  return c.tmax_days > c.tmin_days && c.ngrid_1d > 0 && c.ntstep > 0;
}

bool model_is_finite(const Model &m) {
  // nlte_pops use -1 (no solution yet) and bin W < 0 (no fit): finite sentinels, checked like the rest
  return all_finite(m.level_epsilon, "level_epsilon") && all_finite(m.level_stat_weight, "level_stat_weight") &&
         all_finite(m.phixs_xs, "phixs_xs") && all_finite(m.phixstarget_probability, "phixstarget_probability") &&
         all_finite(m.line_nu, "line_nu") && all_finite(m.line_A, "line_A") && all_finite(m.line_f, "line_f") &&
         all_finite(m.line_coll, "line_coll") && all_finite(m.spontrecombcoeff, "spontrecombcoeff") &&
         all_finite(m.corrphotoioncoeff, "corrphotoioncoeff") && all_finite(m.bfcooling_coeff, "bfcooling_coeff") &&
         all_finite(m.Te, "Te") && all_finite(m.TR, "TR") && all_finite(m.TJ, "TJ") && all_finite(m.W, "W") &&
         all_finite(m.nne, "nne") && all_finite(m.nnetot, "nnetot") && all_finite(m.rho, "rho") &&
         all_finite(m.kappagrey, "kappagrey") && all_finite(m.elem_abundance, "elem_abundance") &&
         all_finite(m.groundlevelpop, "groundlevelpop") && all_finite(m.partfunct, "partfunct") &&
         all_finite(m.totalcooling, "totalcooling") && all_finite(m.cooling_contrib_ion, "cooling_contrib_ion") &&
         all_finite(m.corrphotoionrenorm, "corrphotoionrenorm") && all_finite(m.nlte_pops, "nlte_pops") &&
         all_finite(m.rf_TR, "radfield_bin_TR") && all_finite(m.rf_W, "radfield_bin_W") &&
         all_finite(m.bfrate_est, "bfrate_estimator") && all_finite(m.nt_dep, "nt_deposition_rate_density") &&
         all_finite(m.nt_Y, "nt_ionization_ratecoeff") && all_finite(m.nt_prob, "nt_prob_num_auger") &&
         all_finite(m.nt_ionen, "nt_ionenfrac_num_auger");
}

}  // namespace

extern "C" {

void artis_synth_default_config(artis_synth_config *cfg) {
  std::memset(cfg, 0, sizeof(*cfg));
  cfg->ngrid_1d = 50;
  cfg->nshells_1d = 0;
  cfg->nlevels_per_ion = 400;
  cfg->n_ionising = 56;
  cfg->max_lines = 100000;
  cfg->line_window = 22;
  cfg->n_resonance = 5;
  cfg->ntstep = 50;
  cfg->tmin_days = 3.;
  cfg->tmax_days = 30.;
  cfg->vmax = 1.0e9;
  cfg->mass_msun = 1.0e-4;
  cfg->v_e = 2.7e8;
  cfg->T0 = 1.0e4;
  cfg->n_tclasses = 32;
  cfg->seed = 1281360349ull;
  cfg->ionpot_scale = 1.;
  cfg->thick_tau = 0.;
  cfg->relativistic = 0;
  cfg->instant_particle_deposition = 1;
  cfg->n_kpktdiffusion_timesteps = 0;
  cfg->kpktdiffusion_timescale = 0.;
  cfg->excitation_te = 0;
  cfg->tj_scale = 0.;
  cfg->nebular = 0;
  cfg->nlte_level_max = 80;
  cfg->radfield_nbins = 256;
  cfg->first_nlte_radfield_timestep = 12;
  cfg->detailed_bf_usefromtimestep = 13;
  cfg->minpop = 0.;
  cfg->nu_min_r = 0.;
  cfg->nu_max_r = 0.;
  cfg->grid_spherical = 0;
}

artis_model *artis_model_from_files(const artis_synth_config *cfg, const char *input_txt, const char *model_txt,
                                    const char *abundances_txt) {
  artis_model *m = new artis_model();
  m->cfg = *cfg;
  m->from_files = true;
  artis_ejecta_model em{};
  if (artis_read_input_file(input_txt, &m->inp) != 0 ||
      (m->inp.model_type != 1 && m->inp.model_type != 3) ||
      artis_read_model(model_txt, m->inp.model_type, &em) != 0) {
    delete m;
    return nullptr;
  }
  m->cfg.ntstep = m->inp.ntstep;
  m->cfg.tmin_days = m->inp.tmin_days;
  m->cfg.tmax_days = m->inp.tmax_days;
  if (m->inp.pre_zseed > 0) m->cfg.seed = m->inp.pre_zseed;
  m->cfg.n_kpktdiffusion_timesteps = m->inp.n_kpktdiffusion_timesteps;
  m->cfg.kpktdiffusion_timescale = m->inp.kpktdiffusion_timescale;
  std::mt19937_64 rng(m->cfg.seed);
  build_atomic(*m, rng);
  setup_nebular_atomic(*m);
  std::vector<float> abund((size_t)em.npts_model * m->nelements, 0.f);
  int rc = artis_read_abundances(abundances_txt, em.npts_model, em.model_type, m->nelements, m->elem_anumber.data(),
                                 abund.data());
  if (rc == 0) rc = build_grid_from_model(*m, em, abund);
  artis_free_model(&em);
  if (rc != 0) {
    delete m;
    return nullptr;
  }
  finish_geometry(*m);
  compute_cellstate(*m, 0);
  rebuild_gamma_spectra(*m);
  if (!model_is_finite(*m)) {
    delete m;
    return nullptr;
  }
  return m;
}

artis_model *artis_model_synth(const artis_synth_config *cfg) {
  if (!config_is_sane(*cfg)) return nullptr;
  artis_model *m = new artis_model();
  m->cfg = *cfg;
  std::mt19937_64 rng(cfg->seed);
  build_atomic(*m, rng);
  setup_nebular_atomic(*m);
  build_grid(*m);
  compute_cellstate(*m, 0);
  rebuild_gamma_spectra(*m);
  if (!model_is_finite(*m)) {
    delete m;
    return nullptr;
  }
  return m;
}

void artis_model_free(artis_model *m) { delete m; }
const artis_atomic_tables *artis_model_atomic(const artis_model *m) { return &m->at; }
const artis_geometry *artis_model_geometry(const artis_model *m) { return &m->geom; }
const artis_cell_state *artis_model_cellstate(const artis_model *m) { return &m->cs; }
const artis_te_tables *artis_model_te_tables(const artis_model *m) { return &m->te_tables; }
int64_t artis_model_npts_model(const artis_model *m) { return m->npts_model; }
int artis_model_radfield_nbins(const artis_model *m) { return m->at.radfield_nbins; }
int artis_model_total_nlte_levels(const artis_model *m) { return m->at.total_nlte_levels; }
const int32_t *artis_model_ion_ionstage(const artis_model *m) { return m->at.ion_ionstage; }
void artis_model_ion_ground_statweight(const artis_model *m, float *out) {
  for (int ui = 0; ui < m->at.nions_total; ui++) out[ui] = m->at.level_stat_weight[m->at.ion_uniqueleveloffset[ui]];
}
void artis_model_config(const artis_model *m, artis_synth_config *out) { *out = m->cfg; }

void artis_model_run_params(const artis_model *m, artis_run_params *p) {
  std::memset(p, 0, sizeof(*p));
  p->seed = (uint32_t)m->cfg.seed;
  p->rank = 0;
  p->opacity_case = 4;
  p->do_r_lc = 1;
  p->do_rlc_est = 3;   // test configs: line 9 "4" -> do_rlc_est=3 (input.cc:1976-1979): rlc_emiss_rpkt skipped
  p->n_kpktdiffusion_timesteps = m->cfg.n_kpktdiffusion_timesteps;
  p->kpktdiffusion_timescale = (float)m->cfg.kpktdiffusion_timescale;
  p->max_path_step = 1.e35;  // update_grid.cc:1303 initial value (no cell limits it in this model)
  p->pol_dipole = 1;         // artisoptions_classic.h:64 DIPOLE
  p->relativistic_doppler = m->cfg.relativistic;
  p->record_linestat = 1;
  p->gamma_grey = -1.;       // test configs: "use grey opacity for gammas? -1"
  p->instant_particle_deposition = m->cfg.instant_particle_deposition;
  p->nt_solve_spencerfano = 0;
  p->excitation_temperature = m->cfg.excitation_te ? ARTIS_TEXC_TE : ARTIS_TEXC_TJ;
  p->minpop = minpop_of(*m);
  if (m->cfg.nebular) {  // artisoptions_nltenebular.h
    p->excitation_temperature = ARTIS_TEXC_TE;
    p->nlte_pops_on = 1;
    p->multibin_radfield = 1;
    p->first_nlte_radfield_timestep = m->cfg.first_nlte_radfield_timestep;
    p->detailed_bf_estimators = 1;
    p->detailed_bf_usefromtimestep = m->cfg.detailed_bf_usefromtimestep;
    p->no_lut_photoion = 1;
    p->no_lut_bfheating = 1;
    p->nt_on = 1;
    p->nt_solve_spencerfano = 1;
    p->nt_max_auger_electrons = 2;
    p->pol_dipole = 0;  // DIPOLE undefined (artisoptions_nltenebular.h:68)
  }
  if (m->from_files) {  // input.txt run switches (input.cc:1976-1992, 2013, 2130)
    p->opacity_case = m->inp.opacity_case;
    p->do_r_lc = m->inp.do_r_lc;
    p->do_rlc_est = m->inp.do_rlc_est;
    p->gamma_grey = m->inp.gamma_grey;
  }
}

int artis_model_set_gamma_lines(artis_model *m, int nuc, int nlines, const double *energy_mev, const double *prob) {
  if (nuc < 0 || nuc >= Model::NNUC || nlines < 0 || (nlines > 0 && (!energy_mev || !prob)))
    return ARTIS_ERR_BAD_ARGUMENT;
  m->gl_energy[nuc].assign(energy_mev, energy_mev + nlines);
  m->gl_prob[nuc].assign(prob, prob + nlines);
  rebuild_gamma_spectra(*m);
  return 0;
}

const artis_gamma_spectra *artis_model_gamma_spectra(const artis_model *m) { return &m->gs; }

int artis_model_init_pellets(const artis_model *m, int npkts, uint64_t seed, double etot, double t_model_days,
                             double frac_initial, artis_packet *out) {
  if (npkts <= 0 || !out) return ARTIS_ERR_BAD_ARGUMENT;
  const double t_model = t_model_days * ARTIS_DAY;
  const double wid = 2 * m->geom.coordmax[0] / m->cfg.ngrid_1d;
  // packet_init (packet.cc:77-100): cumulative decay energy per propagation cell, q ~ X(56Ni)(v)
  std::vector<double> cdf(m->ngrid);
  double acc = 0.;
  for (int c = 0; c < m->ngrid; c++) {
    const int mgi = m->cell_mgi[c];
    if (mgi < m->npts_model) {
      const double v = m->mgi_vel[mgi];
      // (vol_init_gridcell x rhoinit x q, packet.cc:99; the uniform grid's equal volumes drop out)
      const double vol = spherical(*m) ? cell_volume(*m, c) : 1.;
      if (m->from_files)
        acc += vol * m->mgi_rho_tmin[mgi] * m->mgi_ni56[mgi];  // model.txt X_Ni56
      else
        acc += vol * m->mgi_rho_tmin[mgi] * 0.6 * exp(-(v / 6e8) * (v / 6e8));
    }
    cdf[c] = acc;
  }
  if (!(acc > 0)) return ARTIS_ERR_BAD_ARGUMENT;
  double share_tot = 0.;
  for (int k = 0; k < kNPath; k++) share_tot += kPath[k].share;
  const double e0 = etot / npkts;
  std::mt19937_64 rng(seed);
  std::uniform_real_distribution<double> U(0., 1.);
  auto upos = [&]() {
    double z;
    do z = U(rng);
    while (z <= 0.);
    return z;
  };
  for (int i = 0; i < npkts; i++) {
    artis_packet p;
    std::memset(&p, 0, sizeof(p));  // packets are calloc'ed (sn3d.cc:816)
    const double r = U(rng) * acc;
    int c = (int)(std::lower_bound(cdf.begin(), cdf.end(), r) - cdf.begin());
    if (c >= m->ngrid) c = m->ngrid - 1;
    while (m->cell_mgi[c] >= m->npts_model) c = (c + 1) % m->ngrid;
    // place_pellet (packet.cc:18-56)
    p.where = c;
    p.number = i;
    p.prop_time = m->tmin;
    p.originated_from_particlenotgamma = 0;
    if (spherical(*m)) {  // a radius uniform in volume within the shell, isotropic direction (packet.cc:29-38)
      const double zrand3 = U(rng);
      const double r_inner = m->cell_pos_min[(size_t)c * 3];
      const double r_outer = r_inner + m->cell_wid[c];
      const double radius = pow(zrand3 * pow(r_inner, 3) + (1. - zrand3) * pow(r_outer, 3), 1 / 3.);
      const double mu = -1 + 2. * U(rng), phi = 2 * ARTIS_PI * U(rng), st = sqrt(1. - mu * mu);
      p.pos[0] = radius * st * cos(phi);
      p.pos[1] = radius * st * sin(phi);
      p.pos[2] = radius * mu;
    } else {
      for (int ax = 0; ax < 3; ax++) p.pos[ax] = m->cell_pos_min[(size_t)c * 3 + ax] + upos() * wid;
    }
    // setup_radioactive_pellet (decay.cc:1371-1458)
    if (U(rng) < frac_initial) {
      p.tdecay = m->tmin;
      p.type = ARTIS_TYPE_RADIOACTIVE_PELLET;
      p.e_cmf = e0;
      p.nu_cmf = e0 / ARTIS_H;
      p.pellet_nucindex = -1;
      p.pellet_decaytype = -1;
    } else {
      const double zc = U(rng) * share_tot;
      int path = 0;
      double cum = 0.;
      for (; path < kNPath - 1; path++) {
        cum += kPath[path].share;
        if (cum > zc) break;
      }
      const PathDef &pd = kPath[path];
      double tdecay = -1;
      while (tdecay <= t_model || tdecay >= m->tmax) {  // sample_decaytime (decay.cc:716-732)
        tdecay = t_model;
        for (int j = 0; j < pd.len; j++) tdecay += -kNuc[pd.nuc[j]].meanlife_d * ARTIS_DAY * log(upos());
      }
      p.tdecay = tdecay;
      p.e_cmf = e0;
      const int nuc = pd.nuc[pd.len - 1];
      p.type = ARTIS_TYPE_RADIOACTIVE_PELLET;
      p.pellet_nucindex = nuc;
      p.pellet_decaytype = pd.decaytype;
      const double e_particle = (pd.decaytype == ARTIS_DECAYTYPE_ELECTRONCAPTURE) ? 0. : kNuc[nuc].e_particle_mev * ARTIS_MEV;
      const double e_gamma = m->gs_endecay[nuc];
      p.originated_from_particlenotgamma = (U(rng) >= e_gamma / (e_gamma + e_particle)) ? 1 : 0;
      p.nu_cmf = e_particle / ARTIS_H;
    }
    const double len = sqrt(p.pos[0] * p.pos[0] + p.pos[1] * p.pos[1] + p.pos[2] * p.pos[2]);
    for (int ax = 0; ax < 3; ax++) p.dir[ax] = p.pos[ax] / len;
    const double t = p.prop_time;
    const double v[3] = {p.pos[0] / t, p.pos[1] / t, p.pos[2] / t};
    double dop = 1. - (p.dir[0] * v[0] + p.dir[1] * v[1] + p.dir[2] * v[2]) / ARTIS_CLIGHT;
    if (m->cfg.relativistic) dop = dop / sqrt(1 - (v[0] * v[0] + v[1] * v[1] + v[2] * v[2]) / ARTIS_CLIGHTSQUARED);
    p.e_rf = p.e_cmf / dop;
    p.trueemissiontype = -1;
    out[i] = p;
  }
  return 0;
}

int artis_model_set_timestep(artis_model *m, int nts) {
  if (nts < 0 || nts >= m->cfg.ntstep) return ARTIS_ERR_BAD_ARGUMENT;
  compute_cellstate(*m, nts);
  return model_is_finite(*m) ? 0 : ARTIS_ERR_BAD_ARGUMENT;
}

// The part of the cell state update_grid does not solve for, at timestep nts: the density rho(t) (the t^-3 expansion
// of grid.cc), the grey opacity and the thick-cell flag; temperatures, populations and cooling are left as they are
// (the timestep loop's update_grid writes them from its solution).  The abundances of the synthetic models do not
// change with time.
int artis_model_advance(artis_model *m, int nts) {
  if (nts < 0 || nts >= m->cfg.ntstep) return ARTIS_ERR_BAD_ARGUMENT;
  Model &mm = *m;
  const double t = mm.ts_mid[nts];
#pragma omp parallel for schedule(static)
  for (int mgi = 0; mgi < mm.npts_model; mgi++) {
    const double rho = mm.mgi_rho_tmin[mgi] * pow(mm.tmin / t, 3);
    if (!(rho > 0)) continue;
    mm.rho[mgi] = (float)rho;
    cell_grey(mm, nts, t, mgi, rho);
  }
  return 0;
}

int artis_model_init_rpackets(const artis_model *m, int nts, int npkts, uint64_t seed, double etot,
                              artis_packet *out) {
  if (nts < 0 || nts >= m->cfg.ntstep || npkts <= 0) return ARTIS_ERR_BAD_ARGUMENT;
  const double t = m->ts_start[nts];
  const int n = m->cfg.ngrid_1d;
  const double wid = 2 * m->geom.coordmax[0] / n;
  // cell CDF by rho * volume (the uniform grid's equal volumes drop out)
  std::vector<double> cdf(m->ngrid);
  double acc = 0.;
  for (int c = 0; c < m->ngrid; c++) {
    const int mgi = m->cell_mgi[c];
    acc += (mgi < m->npts_model) ? m->rho[mgi] * (spherical(*m) ? cell_volume(*m, c) : 1.) : 0.;
    cdf[c] = acc;
  }
  if (!(acc > 0)) return ARTIS_ERR_BAD_ARGUMENT;
  std::mt19937_64 rng(seed);
  std::uniform_real_distribution<double> U(0., 1.);
  for (int i = 0; i < npkts; i++) {
    artis_packet p;
    std::memset(&p, 0, sizeof(p));
    const double r = U(rng) * acc;
    int c = (int)(std::upper_bound(cdf.begin(), cdf.end(), r) - cdf.begin());
    if (c >= m->ngrid) c = m->ngrid - 1;
    while (m->cell_mgi[c] >= m->npts_model) c = (c + 1) % m->ngrid;
    const int mgi = m->cell_mgi[c];
    p.where = c;
    p.type = ARTIS_TYPE_RPKT;
    p.last_cross = ARTIS_NONE;
    if (spherical(*m)) {  // a radius uniform in volume within the shell (away from its faces), isotropic position
      const double z = 0.05 + 0.9 * U(rng);
      const double r_inner = m->cell_pos_min[(size_t)c * 3] * t / m->tmin;
      const double r_outer = (m->cell_pos_min[(size_t)c * 3] + m->cell_wid[c]) * t / m->tmin;
      const double radius = pow(z * pow(r_inner, 3) + (1. - z) * pow(r_outer, 3), 1 / 3.);
      const double pmu = -1 + 2. * U(rng), pphi = 2 * ARTIS_PI * U(rng), pst = sqrt(1. - pmu * pmu);
      p.pos[0] = radius * pst * cos(pphi);
      p.pos[1] = radius * pst * sin(pphi);
      p.pos[2] = radius * pmu;
    } else {
      for (int ax = 0; ax < 3; ax++) {
        const double lo = m->cell_pos_min[(size_t)c * 3 + ax] * t / m->tmin;
        p.pos[ax] = lo + (0.05 + 0.9 * U(rng)) * wid * t / m->tmin;
      }
    }
    const double mu = -1 + 2. * U(rng);
    const double phi = 2 * ARTIS_PI * U(rng);
    const double st = sqrt(1. - mu * mu);
    p.dir[0] = st * cos(phi);
    p.dir[1] = st * sin(phi);
    p.dir[2] = mu;
    // nu_cmf ~ Planck(T_e) in [NU_MIN_R, NU_MAX_R] by rejection (kpkt.cc:428-446)
    const double T = m->Te[mgi];
    const double nu_peak = 5.879e10 * T;
    auto dbb = [&](double nu) { return ARTIS_TWOHOVERCLIGHTSQUARED * pow(nu, 3) / expm1(ARTIS_HOVERKB * nu / T); };
    const double B_peak = dbb(nu_peak);
    double nu;
    while (true) {
      nu = ARTIS_NU_MIN_R + U(rng) * (ARTIS_NU_MAX_R - ARTIS_NU_MIN_R);
      if (U(rng) * B_peak <= dbb(nu)) break;
    }
    p.nu_cmf = nu;
    p.e_cmf = etot / npkts;
    p.prop_time = t;
    const double ndotv = (p.dir[0] * p.pos[0] + p.dir[1] * p.pos[1] + p.dir[2] * p.pos[2]) / t;
    const double dop = 1. - ndotv / ARTIS_CLIGHT;
    p.nu_rf = p.nu_cmf / dop;
    p.e_rf = p.e_cmf / dop;
    p.next_trans = 0;
    p.emissiontype = -1;
    for (int ax = 0; ax < 3; ax++) p.em_pos[ax] = p.pos[ax];
    p.em_time = (int)t;
    p.absorptiontype = 0;
    p.trueemissiontype = -1;
    p.trueem_time = (int)t;
    p.stokes[0] = 1.;
    // pol_dir as emitt_rpkt (rpkt.cc:1009-1022)
    double dd[3] = {0, 0, 1};
    double pd[3] = {p.dir[1] * dd[2] - dd[1] * p.dir[2], p.dir[2] * dd[0] - dd[2] * p.dir[0],
                    p.dir[0] * dd[1] - dd[0] * p.dir[1]};
    if (pd[0] * pd[0] + pd[1] * pd[1] + pd[2] * pd[2] < 1e-8) {
      dd[1] = 1.;
      dd[2] = 0.;
      pd[0] = p.dir[1] * dd[2] - dd[1] * p.dir[2];
      pd[1] = p.dir[2] * dd[0] - dd[2] * p.dir[0];
      pd[2] = p.dir[0] * dd[1] - dd[0] * p.dir[1];
    }
    const double pl = sqrt(pd[0] * pd[0] + pd[1] * pd[1] + pd[2] * pd[2]);
    for (int ax = 0; ax < 3; ax++) p.pol_dir[ax] = pd[ax] / pl;
    p.escape_type = 0;
    p.number = i;
    p.mastate.activatingline = -99;
    p.trueemissionvelocity = -1.f;
    out[i] = p;
  }
  return 0;
}

}  // extern "C"
