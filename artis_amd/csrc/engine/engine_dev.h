// engine_dev.h -- device-side data layout of the MI355X packet-propagation engine.
//
// HBM layout (DESIGN.md "Data layout in HBM"):
//   * packets: structure-of-arrays of the 304-byte reference record viewed as 38 little-endian 8-byte words,
//     soa[word * N + i]; word w of packet i holds bytes [8w, 8w+8) of `struct packet` (packet.h:28-73).
//     A wave touching field f of 64 consecutive packets reads 512 contiguous bytes.
//   * read-only atomic tables uploaded once (artis_gpu_init), plus a per-line record LineTau with the
//     Einstein-B coefficients and unique level indices that get_event needs (rpkt.cc:168-181).
//   * per-cell tables rebuilt per timestep (artis_gpu_upload_cellstate) for the non-empty model cells only,
//     indexed by nonempty index k: level populations, ion-stage populations, departure ratios, cumulative
//     k-packet cooling lists and macro-atom process-rate totals.  These replace the per-OpenMP-thread
//     cellhistory cache (update_grid.cc:659-761) with tables every workitem can read.
#ifndef ARTIS_ENGINE_DEV_H
#define ARTIS_ENGINE_DEV_H

#include <stdint.h>

#define PKT_WORDS 38

// static per-level data of the cached macro-atom walk (two 16-byte loads; the table is L2-resident)
struct __attribute__((aligned(16))) MaMeta {
  int32_t rec_off;     // offset (16-bit keys) of the level's compact record inside a cell's key block
  int32_t doff, uoff;  // level_downtrans_offset, level_uptrans_offset
  int32_t base_lower;  // unique index of level 0 of the next lower ion (-1 if none)
  int32_t nd, nu, nr, nt;  // #downtrans, #uptrans, #recombination targets, #ionisation targets
};

// what one cached-walk step (k_ma's ma_step_cached) reads of a level, with its record layout (ma_layout below) worked
// out on the host: the same two 16-byte loads as MaMeta, and no layout arithmetic (a division by 63 among it) in the
// pass.  w0 = (nd | nu << 16, doff, uoff, base_lower); w1 = (nr | nt << 16, sd | md << 8 | mu << 16 | nbd << 24,
// nbu | end_d << 8 | end_u << 16, hot), end_d / end_u: the line-0 entries of the same-ion searches (separators and
// suffix of a blocked array, else the array)
struct __attribute__((aligned(16))) MaWalk {
  int32_t w[8];
};

// one 32-byte record per line for the line walk of get_event (two 16-byte loads)
struct __attribute__((aligned(16))) LineTau {
  double nu;    // line frequency (linelist_entry.nu)
  double B_ul;  // CLIGHTSQUAREDOVERTWOH / pow(nu, 3) * A_ul          (rpkt.cc:180)
  double B_lu;  // g_u / g_l * B_ul                                    (rpkt.cc:181)
  int32_t ul_lower;  // unique level index of the lower level
  int32_t ul_upper;
};

// per-line constants of the macro-atom rate coefficients, evaluated on the host with the reference expressions
// (so the device never calls pow in the hot loops):  nu_lev = (eps_upper - eps_lower) / H
struct LineMA {
  double B_ul;  // CLIGHTSQUAREDOVERTWOH / pow(nu_lev, 3) * A_ul   (macroatom.cc:521, 565)
  double B_lu;  // g_u / g_l * B_ul                               (macroatom.cc:522, 566)
  double nu3;   // pow(nu_lev, 3)                                 (radfield.h:47)
  double P2;    // pow(H_ionpot / (eps_upper - eps_lower), 2)    (macroatom.h:93, 130)
};

// one collisional-excitation term of get_cooling_ion_coll_exc (kpkt.cc:53-63) at its up-transition index: what
// col_excitation_ratecoeff (macroatom.h:107-150) reads, so a per-line cooling loop is one independent 32-byte load
struct TeExcItem {
  double epsilon_trans;  // epsilon(upper) - epsilon(level)
  double P2;             // LineMA::P2 of the line
  float coll_str, osc_f, upper_sw;
  int32_t forbidden;
};

// k_marates' packed transition items (one 64-byte scalar load per transition, independent of the previous one, so
// the next item and its population are fetched while the current rates are evaluated): what ma_foreach_rate reads of
// a down transition (at level_downtrans_offset + j) and of an up transition (at level_uptrans_offset + j), the same
// values from the same tables (macroatom.cc:57-159 via rad_deexc_core / col_deexc_core / rad_exc_core / col_exc_core)
struct __attribute__((aligned(64))) MaDownItem {
  int32_t lower;      // ion-local index of the lower level
  int32_t forbidden;  // line_forbidden
  float A, coll, osc_f, lower_sw;  // line_einstein_A, line_coll_str, line_osc_strength, stat weight of the lower level
  double eps_target;  // epsilon of the lower level
  double B_ul, B_lu, P2;  // LineMA
};
struct __attribute__((aligned(64))) MaUpItem {
  int32_t upper;      // ion-local index of the upper level
  int32_t forbidden;
  float coll, osc_f, upper_sw, pad;
  double eps_upper;   // epsilon of the upper level
  double B_ul, B_lu, nu3, P2;  // LineMA
};

// one bf continuum's constants for bf_contribution (rpkt.cc:1075-1207), one 32-byte load: its edge, the last
// frequency of its cross-section table (nu_edge * last_phixs_nuovernuedge), probability, table offset
struct BfCont {
  double nu_edge, nu_max, probability;
  int32_t xs_off;  // allcont_phixstable * nphixspoints
  int32_t pad;
};

struct DevTab {
  int32_t nelements, maxnions, nions_total, nlevels_total, nlines, nbf, nbfg, ncoolingterms;
  int32_t nphixspoints, phixs_file_version, tablesize, ntargets_total;
  double nphixsnuincrement, last_phixs_nuovernuedge, mintemp, T_step_log;
  const int32_t *elem_nions, *elem_uniqueionoffset;
  const int32_t *ion_ionstage, *ion_nlevels, *ion_uniqueleveloffset, *ion_ionisinglevels, *ion_maxrecombininglevel,
      *ion_coolingoffset, *ion_ncoolingterms, *ion_element;
  const double *level_epsilon;
  const float *level_stat_weight;
  const int32_t *level_nuptrans, *level_uptrans_offset, *level_ndowntrans, *level_downtrans_offset,
      *level_nphixstargets, *level_phixstargets_offset, *level_cont_index, *level_closestgroundlevelcont,
      *level_phixstable, *level_ui;
  const int32_t *uptrans_lineindex, *downtrans_lineindex, *phixstarget_levelindex;
  const double *phixstarget_probability;
  const float *phixs_xs;
  const double *line_nu;
  const double *line_nu8;  // line_nu padded with zeros to a multiple of 8 (64-byte windows of the line walk)
  const float *line_A, *line_f, *line_coll;
  const int32_t *line_elem, *line_ion, *line_upper, *line_lower;
  const uint8_t *line_forbidden;
  const LineTau *line_tau;
  const LineMA *line_ma;
  const TeExcItem *exc_items;  // [sum nuptrans] indexed like uptrans_lineindex (k_cooling, k_te_solve)
  const MaDownItem *ma_down;  // [sum ndowntrans] indexed like downtrans_lineindex (k_marates)
  const MaUpItem *ma_up;      // [sum nuptrans] indexed like uptrans_lineindex (k_marates)
  // per level: offset (doubles) of its macro-atom record inside a cell's record block, #downtrans, #uptrans,
  // #recombination targets (ionising levels of the lower ion, 0 if the level does not recombine)
  const MaMeta *ma_meta;  // [nlevels_total]
  const MaWalk *ma_walk;  // [nlevels_total]
  const int64_t *ma_dbl_off;  // [nlevels_total + 1] offset (doubles) of each level's exact record in k_marates' scratch
  // targets of the internal same-ion jumps in the order of their level's cumulative arrays (downtrans / uptrans
  // order): (unique level index, offset of its macro-atom record in a cell block)
  const int2 *down_target, *up_target;
  const double *allcont_nu_edge, *allcont_probability;
  const BfCont *bfc;  // [nbf]
  const double2 *bf_edge2;  // [nbf rounded up past a multiple of 4] {nu_edge, nu_max}, padded with infinities
                            // (transport.h bf_range)
  const int32_t *allcont_element, *allcont_ion, *allcont_level, *allcont_target, *allcont_upperlevel,
      *allcont_phixstable, *allcont_groundindex;
  const double *groundcont_nu_edge;
  const int32_t *groundcont_element, *groundcont_ion;
  const int32_t *gc_cont_off, *gc_cont;  // per ground continuum: its ground-level allcont indices (CSR, ascending)
  const double *spontrecombcoeff, *corrphotoioncoeff, *bfcooling_coeff;
  const int32_t *cool_type, *cool_element, *cool_ion, *cool_level, *cool_upper;
  // nebular options (ABI 6): NLTE level bookkeeping (input.cc:1711-1746), radiation-field bin edges
  // (radfield.cc:131-188), the allcont index of each photoionisation target slot (get_bfcontindex)
  const int32_t *ion_nlevels_nlte, *ion_first_nlte;
  int32_t total_nlte_levels, rf_nbins;
  const double *rf_nu_upper;
  double rf_nu_lower_first;
  const int32_t *slot_allcont;
  // gamma-ray line spectra per nuclide (gammapkt.cc:27-33), uploaded by artis_gpu_init_gamma
  int32_t g_nnuc;
  const int32_t *g_nlines, *g_off;
  const double *g_endecay, *g_energy, *g_prob;
  int32_t g_nsorted;             // allnuc_gamma_line_list size (gammapkt.cc:192-211)
  const double *g_freq_sorted;   // its frequencies (get_gam_freq, gammapkt.cc:702-718) in list order
};

// Record layout of the macro-atom key cache (DevCells::ma_key), in 16-bit key positions.  k_ma stages one 128-byte
// line (64 positions) of a record per lane and pass, so the layout puts what most jumps need on the first line:
//   line 0:  [0, 9) the action keys | [9, 9 + sd) down-same area | [9 + sd, 9 + sd + su) up-same area
//   lines 1 .. nbd:            the down-same keys before the area's suffix in 64-key blocks (if it overflows the area)
//   lines nbd + 1 .. nbd+nbu:  the up-same keys likewise
//   from line 1 + nbd + nbu:   rad_deexc (nd) | rad_recomb (nr) | internal_down_lower (nr) | internal_up_higher (nt)
// then the low halves of all positions (offset `hot`).  A same-ion array that fits its area (most levels) is
// stored there whole.  One that does not keeps the last key of every block (separators) there, followed by its last
// md / mu keys (the suffix): separators and suffix are one ascending sequence, so a search of line 0 either ends in
// the suffix (one pass) or names the block that holds the key (a second pass).  The suffix is what a blocked array's
// share of line 0 adds to the layout of round 4 (separators only: every search of such an array took two passes,
// 38 % of the up-same searches of the bench).  A suffix, because these are the low levels' upward arrays, and the
// selections fall at their ends (stamps build, profiles/r5p1_stamps.txt: 80 % in the last quarter of arrays of
// ~400 keys, 30 % in the last 48 keys; 0.0002 % in the first 48).  The 55 area slots go to whichever array needs them.
#ifndef ARTIS_MA_SUFFIX
#define ARTIS_MA_SUFFIX 1
#endif
struct MaLayout {
  int sd, su;    // line-0 slots of the down / up array (its keys, or its block separators and suffix)
  int nbd, nbu;  // 64-key blocks of the down / up array outside line 0 (0: the array is on line 0)
  int md, mu;    // keys of the down / up array stored whole on line 0 (the array's size if it fits)
  int sorted0;   // record position of the first rad_deexc key
  int hot;       // high-half positions = offset of the low halves
};
// blocks of an array of c keys whose line-0 area has s slots, and its line-0 suffix *m (negative: does not fit)
static inline __host__ __device__ int ma_blocks(int c, int s, int *m) {
  if (c <= s) {
    *m = c;
    return 0;
  }
#if ARTIS_MA_SUFFIX
  // nb blocks of 64 and a suffix of s - nb keys: the least nb with 64 nb + s - nb >= c
  const int nb = (c - s + 62) / 63;
#else
  const int nb = (c + 63) / 64;  // (round 4: the separators of all blocks but the last, no suffix)
  if (nb - 1 > s) {
    *m = -1;
    return nb;
  }
#endif
  *m = ARTIS_MA_SUFFIX ? s - nb : 0;
  return nb;
}
// k_rpkt's per-block estimator accumulator (few-cell models: every update of the same few addresses would otherwise
// serialise in the memory system's atomics)
#define EST_LDS_DOUBLES 2048
#define MA_AREA 55
// level mode: the records hold the high key halves only (twice the records in the same pool; a comparison the high
// half cannot decide is made from the exact sums by k_ma's cooperative jump)
#ifndef ARTIS_MA_HI_ONLY
#define ARTIS_MA_HI_ONLY 1
#endif
#define MA_NOLINE 0xffffffffu  // DevCells::ma_lptr: no record for this (cell, level)
static inline __host__ __device__ MaLayout ma_layout(int nd, int nu, int nr, int nt) {
  MaLayout L;
  if (nd + nu <= MA_AREA) {
    L.sd = nd;
    L.su = nu;
  } else if (nd <= MA_AREA / 2) {
    L.sd = nd;
    L.su = MA_AREA - nd;
  } else if (nu <= MA_AREA / 2) {
    L.su = nu;
    L.sd = MA_AREA - nu;
  } else {
    L.sd = MA_AREA / 2;
    L.su = MA_AREA - MA_AREA / 2;
  }
  L.nbd = ma_blocks(nd, L.sd, &L.md);
  L.nbu = ma_blocks(nu, L.su, &L.mu);
  L.sorted0 = 64 * (1 + L.nbd + L.nbu);
  L.hot = L.sorted0 + nd + 2 * nr + nt;
  return L;
}
// separators on line 0 of a blocked array of nb blocks
static inline __host__ __device__ int ma_nsep(int nb) { return ARTIS_MA_SUFFIX ? nb : nb - 1; }
// the level's MaWalk record; false if a field does not fit its bits
static inline __host__ __device__ bool ma_walk_make(const MaMeta &m, MaWalk *w) {
  const MaLayout L = ma_layout(m.nd, m.nu, m.nr, m.nt);
  const int end_d = L.nbd ? ma_nsep(L.nbd) + L.md : m.nd, end_u = L.nbu ? ma_nsep(L.nbu) + L.mu : m.nu;
  const bool ok = m.nd < 65536 && m.nu < 65536 && m.nr < 65536 && m.nt < 65536 && L.sd < 256 && L.md >= 0 &&
                  L.md < 256 && L.mu >= 0 && L.mu < 256 && L.nbd < 256 && L.nbu < 256 && end_d < 256 && end_u < 256 &&
                  L.sorted0 < 65536;
  w->w[0] = m.nd | (m.nu << 16);
  w->w[1] = m.doff;
  w->w[2] = m.uoff;
  w->w[3] = m.base_lower;
  w->w[4] = m.nr | (m.nt << 16);
  w->w[5] = L.sd | (L.md << 8) | (L.mu << 16) | (L.nbd << 24);
  w->w[6] = L.nbu | (end_d << 8) | (end_u << 16);
  w->w[7] = L.hot;
  return ok;
}
// a blocked array needs one separator slot per block but the last beside its prefix
static inline __host__ __device__ bool ma_layout_ok(int nd, int nu) {
  const MaLayout L = ma_layout(nd, nu, 0, 0);
  return L.md >= 0 && L.mu >= 0;
}
// key j of a same-ion array of c keys (area at a0, suffix m, nb blocks from record line lb): its record position;
// *sep the separator position on line 0 the key is also stored at, or -1
static inline __host__ __device__ int ma_same_pos(int j, int c, int a0, int m, int nb, int lb, int *sep) {
  if (!nb) return a0 + j;
  const int cb = c - m;  // keys in the blocks
  if (j >= cb) return a0 + ma_nsep(nb) + (j - cb);
  if (((j & 63) == 63 || j == cb - 1) && (j >> 6) < ma_nsep(nb)) *sep = a0 + (j >> 6);
  return 64 * (lb + (j >> 6)) + (j & 63);
}
// record position of scratch position p (k_marates order: [9 totals | down nd | up nu | the sorted arrays])
static inline __host__ __device__ int ma_rec_pos(const MaLayout &L, int p, int nd, int nu, int *sep) {
  *sep = -1;
  if (p < 9) return p;
  if (p < 9 + nd) return ma_same_pos(p - 9, nd, 9, L.md, L.nbd, 1, sep);                               // down-same
  if (p < 9 + nd + nu) return ma_same_pos(p - 9 - nd, nu, 9 + L.sd, L.mu, L.nbu, 1 + L.nbd, sep);  // up-same
  return L.sorted0 + (p - 9 - nd - nu);
}

struct DevGeom {
  int32_t ncoordgrid[3];
  int32_t ngrid, npts_model;
  int32_t spherical;        // GRID_SPHERICAL1D (boundary.cc:136-140, 234-244): radial shells, cellindex == mgi
  const double *cell_pos_min;
  const double *cell_wid;   // [ngrid] wid_init(cellindex) of the spherical grid (grid.cc:76-91); nullptr otherwise
  const int32_t *cell_mgi;
  double coordmax0, tmin, rmax, wid, tmax, vmax;
  const double *ts_start, *ts_width, *ts_mid;
  double nu_min_r, nu_max_r;
};

struct DevCells {
  const float *Te, *TR, *TJ, *W, *nne, *nnetot, *rho, *kappagrey;
  const int16_t *thick;
  const float *elem_abundance, *groundlevelpop, *partfunct;
  const double *totalcooling, *cooling_contrib_ion, *corrphotoionrenorm;
  const float *ffegrp;      // [npts_model] or nullptr (gamma opacities, photo_electric.cc:34)
  const int32_t *ne_index;  // [npts_model] nonempty index, -1 if the model cell is empty
  const int32_t *ne_mgi;    // [n_nonempty]
  int32_t n_nonempty;
  double *pops;        // [n_nonempty * nlevels_total]  calculate_levelpop (ltepop.cc:417-430)
  double *ionpop;      // [n_nonempty * nions_total]    ionstagepop (ltepop.cc:558-564)
  double *ffsum;       // [n_nonempty]                  sum_ions Z^2 n_ion of calculate_kappa_ff (rpkt.cc:1036-1058)
  // per (cell, continuum) {n_level if the continuum is included in the cell's kappa_bf (rpkt.cc:1116-1118) else 0,
  // departure ratio (rpkt.cc:1140-1151)}: bf_contribution's cell data in one 16-byte load, no index chain
  double2 *bfcell;     // [n_nonempty * nbf]
  double *corrphot;    // [n_nonempty * ntargets_total] get_corrphotoioncoeff (ratecoeff.cc:1247-1308)
  // level-major copies for k_marates, whose lanes run over consecutive cells of one level (coalesced reads)
  double *popsT;       // [nlevels_total * n_nonempty]
  double *corrphotT;   // [ntargets_total * n_nonempty]
  double *cooling;     // [n_nonempty * ncoolingterms]  cumulative cooling_contrib (kpkt.cc:167-308)
  // Sobolev coefficient of every line in every cell, (B_lu n_l - B_ul n_u) * HCLIGHTOVERFOURPI (rpkt.cc:168-187;
  // tau_line = coefficient * t), rows padded to linecoef_stride = nlines rounded up to 8, for the first
  // linecoef_rows non-empty cells (the HBM budget's share; the line walk of a cell k >= linecoef_rows gathers the
  // two populations per line itself); nullptr when no row fits
  double *linecoef;    // [linecoef_rows * linecoef_stride]
  int64_t linecoef_stride;
  int32_t linecoef_rows;
  int32_t *linecoef_neg;  // [1]: k_linecoef found a negative coefficient (a population inversion) in some row
  // macro-atom cache: per (cell, level) one compact record of 32-bit keys, 128-byte aligned.  A key is a running
  // sum of the reference's individual rates (the cellhistory individ_* arrays, globals.h:174-183, summed in the
  // reference's order, macroatom.cc:57-159) divided by its action's total and rounded to 32 bits; the first 9 are
  // the running sums of the 9 process-rate totals over their grand total.  The keys' high halves come first (the
  // hot part: a typical jump reads one 128-byte line of them) and their low halves after (read only when the high
  // half cannot decide a comparison).  A search compares the uniform draw with the keys; a key within rounding of
  // the draw leaves the comparison undecided and the jump is made with the exact sums (ma_jump_exact) -- the
  // selections are the reference's linear-scan choices either way.  The two arrays of the internal same-ion
  // jumps (most jumps) come first, in Eytzinger (BFS) order, their top entries on the record's first line
  // (ma_rec_pos above):
  //   [9 action keys | internal_down_same (nd, Eytzinger) | internal_up_same (nu, Eytzinger) | rad_deexc (nd) |
  //    rad_recomb (nr) | internal_down_lower (nr) | internal_up_higher (nt)]  high halves, then the same
  //   positions' low halves; the record padded to a multiple of 64 keys
  uint16_t *ma_key;    // [n_nonempty * ma_key_stride], or nullptr
  int64_t ma_key_stride;
  int32_t have_macache;  // ma_rows > 0
  // row mode: every non-empty cell's records, cell k's at row ma_row[k] (the records of one cell are contiguous,
  // the level's at MaMeta::rec_off).  ma_bin[k] is cell k's bin in the binned M queue (centre outwards).
  int32_t ma_rows;
  const int32_t *ma_row;  // [n_nonempty]
  const int32_t *ma_bin;  // [n_nonempty]
  // level mode (the records of every cell do not fit the budget, ma_rows == 0): records per (cell, level) in the
  // pool ma_key, for the pairs the walks used most in the previous timestep (engine.hip ma_level_place);
  // ma_lptr[k * nlevels_total + ul] is the first 128-byte line of the record, MA_NOLINE for a pair without one
  // (k_ma evaluates its rates with the whole wave, ma_coop_select); ma_lhist counts the jumps per pair: a cached
  // jump is sampled (every 16th jump of a walk adds 16), an exact-sum jump adds 1 (it is made by the whole wave over
  // the level's rate list, so its one atomic is a small part of it, and the pairs without a record -- the ones the
  // next placement must find -- are counted exactly)
  const uint32_t *ma_lptr;  // [n_nonempty * nlevels_total] or nullptr (row mode)
  uint32_t *ma_lhist;       // [n_nonempty * nlevels_total] or nullptr
  // few-cell models: offsets (doubles) of the J / nuJ / ffheating, bfrate and radfield-bin estimators of every
  // non-empty cell in k_rpkt's LDS accumulator (EST_LDS_DOUBLES), -1 where they do not fit (per-lane atomics)
  int32_t est_lds_J, est_lds_bf, est_lds_rf;
  int32_t ma_level_mode;
  int32_t ma_hi_only;  // the records hold the high key halves only (level mode): a comparison that needs the low
                       // half is undecided and the jump goes to k_ma_exact
  double *marates;     // level mode: [n_nonempty * nlevels_total * 9] the per-pair action totals (or nullptr)
  // nebular inputs (ABI 6; nullptr when the option is off), model-cell indexed like the arrays above
  const double *nlte_pops;    // [npts_model * total_nlte_levels]
  const float *rf_TR, *rf_W;  // [npts_model * rf_nbins]
  const float *bfrate_est;    // [npts_model * nbf]
  const double *nt_dep;       // [npts_model]
  const double *nt_Y;         // [npts_model * nions_total]
  const float *nt_prob, *nt_ionen;  // [npts_model * nions_total * (nt_max_auger + 1)]
  // derived per non-empty cell (k_ntcells): running sums of ion_ntion_energyrate over (element, lower ion) in
  // select_nt_ionization2 order, at the unique index of the lower ion (nonthermal.cc:1827-1875), and their total
  double *nt_cum;             // [n_nonempty * nions_total]
  double *nt_total;           // [n_nonempty]
};

struct DevEst {
  double *J, *nuJ, *ffheat, *colheat, *rpkt_emiss, *gamma, *bfheat;  // contiguous block, see engine.hip
  double *bfrate;                  // [npts_model * nbf] bfrate_raw (DETAILED_BF_ESTIMATORS_ON), in the block
  double *rfJ, *rfnuJ, *rfcount;   // [npts_model * rf_nbins] radfield bin estimators (contribcount as double)
  double *compton;                 // [(npts_model + 1) * ARTIS_EMISS_MAX] compton_emiss (ABI 10), in the block
  int32_t *ecounter, *acounter;
  double *scalars;                 // [10] cmf_lum, gamma_dep, ... (artis_estimators order), nt_energy_deposited,
                                   // pellet_decays
  unsigned long long *counters;    // [34] + nesc at [34]
  unsigned long long *work;        // [16]
  int32_t *err;                    // [4] code, packet number, aux, aux
};

// virtual packets (VPKT_ON, vpkt.cc): parameters of artis_vpkt_params, derived bins, accumulators, and the spawn
// buffer the emission sites append to (vpkt.h)
#define VPKT_MAX_SPECTRA 8
#define VPKT_MRANGE 4
#define VPKT_MRANGE_GRID 5
#define VPKT_SPAWN_WORDS 13
struct DevVpkt {
  int32_t on;
  int32_t nobs, nspectra, vmtbins, vmnubins, nrange, vgrid_flag, nrange_grid, ny_vgrid, nz_vgrid, nprocs;
  double exclude[VPKT_MAX_SPECTRA];
  double tmin_vspec, tmax_vspec, numin_vspec, numax_vspec, dlogt, dlognu;
  double tmin_input, tmax_input, numin_input[VPKT_MRANGE], numax_input[VPKT_MRANGE];
  double tau_max;
  double tmin_grid, tmax_grid, nu_grid_min[VPKT_MRANGE_GRID], nu_grid_max[VPKT_MRANGE_GRID];
  const double *obs;        // [nobs * 3] observer unit vectors (host libm, vpkt.cc:863-865)
  const float *delta_t;     // [vmtbins]  vspecpol.delta_t (float, vpkt.cc:18)
  const float *delta_freq;  // [vmnubins] delta_freq_vspec (float, vpkt.cc:26)
  const int32_t *anumber;   // [nelements]
  const uint8_t *line_mask; // [nlines padded to 8 + 8] bit ind: the line's opacity enters spectrum ind
  double *vstokes;          // [3][vmtbins][nobs * nspectra][vmnubins]: I, Q, U
  int64_t vstokes_stride;   // doubles per Stokes component
  double *vgrid;            // [3][ny][nz][nrange_grid][nobs]
  int64_t vgrid_stride;
  unsigned long long *ctr;  // [8]: nvpkt, nvpkt_esc1..3, traces, cell segments, lines scanned, spawns dropped
  // spawn records, word-major: spawn[w * cap + s]; words: 0-2 pos, 3-5 dir, 6 nu_cmf, 7 e_cmf, 8-9 stokes Q, U,
  // 10 prop_time (= t_current at every call site), 11 (where, next_trans), 12 (last_cross, realtype)
  double *spawn;
  uint32_t *spawn_ctr;      // [2]: appended, trace fetch head
  uint32_t cap;
  // a full buffer: the spawn that found it full goes to the overflow records (same word-major layout, stride
  // ovf_cap) and sets *full; k_rpkt / k_kpkt then take no new packets, k_rpkt parks each packet at its first
  // overflow, and the host traces the buffer, moves the overflow records to its front and resumes the launch
  // (engine.hip vpkt_drain).  ovf_cap covers one overflow per resident lane.
  double *ovf;
  // trace order: k_vpkt takes its work items observer-major over the spawns sorted by (propagation cell, log nu)
  // (perm[j]: the j-th spawn in that order; nullptr: buffer order), so a wave traces parallel paths from one cell
  // at nearby frequencies -- the same cells, linecoef rows and line windows
  const uint32_t *perm;
  uint32_t *ovf_ctr;        // [1]
  uint32_t *full;           // [1]
  uint32_t ovf_cap;
  // the coefficient table has a negative entry (DevCells::linecoef_neg, read back after the precompute): only then
  // can a virtual packet's tau fall along a line walk over it (vpkt_trace_segment's per-line check)
  int32_t neg_coef;
};

struct DevRun {
  uint32_t seed;
  int32_t rank;
  int32_t opacity_case, do_r_lc, do_rlc_est, n_kpktdiffusion_timesteps;
  float kpktdiffusion_timescale;
  double max_path_step;
  int32_t pol_dipole, relativistic_doppler, record_linestat;
  double gamma_grey;
  int32_t instant_particle_deposition, nt_solve_spencerfano;
  int32_t exc_te;  // 1: level populations at T_e (LTEPOP_EXCITATIONTEMPERATURE), 0: at T_J
  double minpop;   // MINPOP
  int32_t nts;     // timestep of the uploaded cell state (globals::nts_global for radfield / get_corrphotoioncoeff)
  int32_t nlte_on, multibin, first_nlte_rf, detailed_bf, detailed_bf_usefrom, no_lut_photoion, no_lut_bfheating;
  int32_t nt_on, nt_max_auger;
  // ABI 10: Compton / pair-production emissivity estimators (emissivities.cc:14-136)
  int32_t comp_est;      // the caller's switch (artis_run_params.comp_est)
  int32_t comp_est_now;  // do_comp_est of the timestep being propagated (sn3d.cc:539, estim_switch)
  int32_t emiss_offset, emiss_max;
  double time_syn_first, time_syn_last;
  double syn_dir[3];
};

#endif
