// engine.hip -- MI355X (gfx950) packet-propagation engine behind the C-ABI of include/artis_gpu.h.
//
// Per timestep:
//   artis_gpu_upload_cellstate: H2D of the update_grid outputs, then five precompute kernels over the
//     non-empty model cells (populations, ion-stage pops + free-free ion sums, departure ratios, corrected
//     photoionisation coefficients, cumulative k-packet cooling lists, macro-atom process-rate totals) --
//     the GPU replacement of the per-thread cellhistory cache (update_grid.cc:659-761).
//   artis_gpu_update_packets: H2D of the 304-byte packet records, AoS->SoA transpose, the transport kernel
//     (one packet per workitem, update_packets.cc:234-333 with the pass loop flattened), SoA->AoS, D2H, and
//     the estimator sums added into the caller's arrays.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <rccl/rccl.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <map>
#include <type_traits>
#include <vector>

#include "artis_constants.h"
#include "artis_gpu.h"
#include "artis_rng.h"
#include "engine_dev.h"
#include "packet_soa.h"
#include "physics.h"
#include "transport.h"
#include "wavefront.h"
#include "spectrum.h"
#include "vpkt.h"
#include "qag.h"
#include "te_solver.h"
#include "nlte_solver.h"

// ================================================================================================= kernels

// ltepop.cc:307-347,417-430,558-564; rpkt.cc:1036-1058 (free-free ion sum)
__global__ void k_cellprep(Ctx K) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= K.C.n_nonempty) return;
  const int mgi = K.C.ne_mgi[k];
  double ffsum = 0.;
  for (int e = 0; e < K.T.nelements; e++) {
    for (int i = 0; i < K.T.elem_nions[e]; i++) {
      const int ui = uion(K, e, i);
      double gp = K.C.groundlevelpop[(int64_t)mgi * K.T.nions_total + ui];
      if (gp < K.R.minpop) gp = (K.C.elem_abundance[(int64_t)mgi * K.T.nelements + e] > 0) ? K.R.minpop : 0.;
      const double nnion = gp * K.C.partfunct[(int64_t)mgi * K.T.nions_total + ui] /
                           (double)K.T.level_stat_weight[K.T.ion_uniqueleveloffset[ui]];
      K.C.ionpop[(int64_t)k * K.T.nions_total + ui] = nnion;
      const int Z = K.T.ion_ionstage[ui] - 1;
      if (Z > 0) ffsum += Z * Z * 1. * nnion;
    }
  }
  K.C.ffsum[k] = ffsum;
}

__global__ void k_levelpops(Ctx K) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nl = K.T.nlevels_total;
  if (idx >= (int64_t)K.C.n_nonempty * nl) return;
  const int k = (int)(idx / nl);
  const int ul = (int)(idx % nl);
  const int mgi = K.C.ne_mgi[k];
  const int ui = K.T.level_ui[ul];
  const int e = K.T.ion_element[ui];
  const int l = ul - K.T.ion_uniqueleveloffset[ui];
  const int ul0 = K.T.ion_uniqueleveloffset[ui];
  const bool hasabund = K.C.elem_abundance[(int64_t)mgi * K.T.nelements + e] > 0;
  const double minpop = K.R.minpop;
  double ng = K.C.groundlevelpop[(int64_t)mgi * K.T.nions_total + ui];
  if (ng < minpop) ng = hasabund ? minpop : 0.;
  const double T_exc = K.R.exc_te ? K.C.Te[mgi] : K.C.TJ[mgi];  // ltepop.cc:338
  double nn;
  if (l == 0) {
    nn = ng;
  } else {
    if (K.R.nlte_on) {
      // ltepop.cc:349-415: NLTE levels 1..nlevels_nlte and the superlevel (nltepop.cc:1543-1554), unless the
      // stored value marks "no NLTE solution yet" (< -0.9)
      const int nn_nlte = K.T.ion_nlevels_nlte[ui];
      const double *row = K.C.nlte_pops + (int64_t)mgi * K.T.total_nlte_levels + K.T.ion_first_nlte[ui];
      const double rho = K.C.rho[mgi];
      if (l <= nn_nlte) {
        const double v = row[l - 1];
        if (!(v < -0.9)) {
          K.C.pops[idx] = v * rho;
          return;
        }
      } else {
        const double v = row[nn_nlte];
        if (!(v < -0.9)) {
          const int sl = ul0 + nn_nlte + 1;
          const double boltz = (double)K.T.level_stat_weight[ul] / (double)K.T.level_stat_weight[sl] *
                               exp(-(K.T.level_epsilon[ul] - K.T.level_epsilon[sl]) / ARTIS_KB / T_exc);
          K.C.pops[idx] = v * rho * boltz;
          return;
        }
      }
    }
    const double W = 1.;
    nn = (ng * W * (double)K.T.level_stat_weight[ul] / (double)K.T.level_stat_weight[ul0] *
          exp(-(K.T.level_epsilon[ul] - K.T.level_epsilon[ul0]) / ARTIS_KB / T_exc));
  }
  if (nn < minpop) nn = hasabund ? minpop : 0.;
  K.C.pops[idx] = nn;
}

// rpkt.cc:1140-1151 departure ratios; ratecoeff.cc:1247-1308 corrected photoionisation coefficients
__global__ void k_bfcells(Ctx K, const int32_t *target_ul, const int32_t *target_t) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nb = K.T.nbf, ntg = K.T.ntargets_total;
  const int64_t total = (int64_t)K.C.n_nonempty * (nb + ntg);
  if (idx >= total) return;
  const int k = (int)(idx / (nb + ntg));
  const int r = (int)(idx % (nb + ntg));
  const int mgi = K.C.ne_mgi[k];
  const double *pops = K.C.pops + (int64_t)k * K.T.nlevels_total;
  if (r < nb) {
    const int i = r;
    const int element = K.T.allcont_element[i];
    const int ion = K.T.allcont_ion[i];
    const int level = K.T.allcont_level[i];
    const int upper = K.T.allcont_upperlevel[i];
    const double T_e = K.C.Te[mgi];
    const double nne = K.C.nne[mgi];
    const double nnlevel = pops[ulev(K, element, ion, level)];
    const double nnupperionlevel = pops[ulev(K, element, ion + 1, upper)];
    const double sf = calculate_sahafact(K, element, ion, level, upper, T_e, ARTIS_H * K.T.allcont_nu_edge[i]);
    // bf_contribution's inclusion rule (rpkt.cc:1116-1118): DETAILED_BF_ESTIMATORS_ON includes every continuum of
    // an element present in the cell, otherwise the ion must hold > 1e-6 of the cell's nuclei (or the level is the
    // ground level)
    const double depratio = nnupperionlevel / nnlevel * nne * sf;
    if (!K.C.ionpop) {
      // the nebular update_grid's context (artis_gpu_update_grid_nlte): no ion populations of its active cells, and
      // only the departure ratio is read there
      K.C.bfcell[(int64_t)k * nb + i].y = depratio;
      return;
    }
    const int ui = uion(K, element, ion);
    const bool incl = K.R.detailed_bf
                          ? K.C.elem_abundance[(int64_t)mgi * K.T.nelements + element] > 0
                          : ((K.C.ionpop[(int64_t)k * K.T.nions_total + ui] / (double)K.C.nnetot[mgi] > 1.e-6) || level == 0);
    K.C.bfcell[(int64_t)k * nb + i] = make_double2(incl ? nnlevel : 0., depratio);
  } else {
    const int slot = r - (int)nb;
    const int ul = target_ul[slot];
    const int t = target_t[slot];
    const int ui = K.T.level_ui[ul];
    const int e = K.T.ion_element[ui];
    const int i = ui - K.T.elem_uniqueionoffset[e];
    const int l = ul - K.T.ion_uniqueleveloffset[ui];
    // ratecoeff.cc:1255-1261: the previous timestep's bf-rate estimator when there is one
    if (bfrate_override(K, mgi, slot)) {
      K.C.corrphot[(int64_t)k * ntg + slot] = K.C.bfrate_est[(int64_t)mgi * K.T.nbf + K.T.slot_allcont[slot]];
      return;
    }
    if (K.R.no_lut_photoion) return;  // k_corrphot_integral
    const double W = K.C.W[mgi];
    const double T_R = K.C.TR[mgi];
    double gammacorr = W * lut_interp(K, K.T.corrphotoioncoeff, e, i, l, t, T_R);
    const int g = K.T.level_closestgroundlevelcont[ul];
    if (g >= 0) gammacorr *= K.C.corrphotoionrenorm[(int64_t)mgi * K.T.nelements * K.T.maxnions + g];
    K.C.corrphot[(int64_t)k * ntg + slot] = gammacorr;
  }
}

// nonthermal.cc:1827-1875 per non-empty cell: ion_ntion_energyrate of every (element, lower ion) summed in
// select_nt_ionization2's order (running sums at the lower ion's unique index, total = get_ntion_energyrate)
__global__ void k_ntcells(Ctx K) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= K.C.n_nonempty) return;
  const int mgi = K.C.ne_mgi[k];
  const int ni = K.T.nions_total;
  double *cum = K.C.nt_cum + (int64_t)k * ni;
  double ratesum = 0.;
  for (int e = 0; e < K.T.nelements; e++) {
    const int nions = K.T.elem_nions[e];
    for (int lowerion = 0; lowerion < nions; lowerion++) {
      const int ui = uion(K, e, lowerion);
      if (lowerion < nions - 1) {
        const double nnlowerion = K.C.ionpop[(int64_t)k * ni + ui];
        double enrate = 0.;
        for (int upperion = lowerion + 1; upperion <= nt_ionisation_maxupperion(K, e, lowerion); upperion++) {
          const double upperionprobfrac = nt_ionization_upperion_probability(K, mgi, e, lowerion, upperion, false);
          const double epsilon_trans = epsilon(K, e, upperion, 0) - epsilon(K, e, lowerion, 0);
          enrate += nnlowerion * upperionprobfrac * epsilon_trans;
        }
        ratesum += K.C.nt_Y[(int64_t)mgi * ni + ui] * enrate;
      }
      cum[ui] = ratesum;
    }
  }
  K.C.nt_total[k] = ratesum;
}

// kpkt.cc:167-308 calculate_kpkt_rates_ion, one workitem per (cell, ion), cumulative from oldcoolingsum.
// Workitems are ion-major (consecutive lanes = the same ion in consecutive cells), as k_marates: the lanes of a wave
// walk the same level and transition lists (uniform loads, no divergence) and read the populations from the
// level-major copy popsT (coalesced).
__global__ void k_cooling(Ctx K) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int ni = K.T.nions_total;
  const int64_t nne_cells = K.C.n_nonempty;
  if (idx >= nne_cells * ni) return;
  const int ui = (int)(idx / nne_cells);
  const int k = (int)(idx % nne_cells);
  const int mgi = K.C.ne_mgi[k];
  const int e = K.T.ion_element[ui];
  const int i = ui - K.T.elem_uniqueionoffset[e];
  const float nne = K.C.nne[mgi];
  const float T_e = K.C.Te[mgi];
  const double *popsT = K.C.popsT + k;  // popsT[u * nne_cells]: level u of this lane's cell
  double *cc = K.C.cooling + (int64_t)k * K.T.ncoolingterms;
  double oldcoolingsum = 0.;
  for (int u = 0; u < ui; u++) oldcoolingsum += K.C.cooling_contrib_ion[(int64_t)mgi * ni + u];
  double contrib = oldcoolingsum;
  int idxc = K.T.ion_coolingoffset[ui];
  const int nions = K.T.elem_nions[e];
  const int nlevels = K.T.ion_nlevels[ui];
  const int ionisinglevels = K.T.ion_ionisinglevels[ui];
  const double nncurrention = K.C.ionpop[(int64_t)k * ni + ui];
  const int ioncharge = K.T.ion_ionstage[ui] - 1;
  if (ioncharge > 0) {
    const double C = 1.426e-27 * sqrt((double)T_e) * pow((double)ioncharge, 2) * nncurrention * nne;
    contrib += C;
    cc[idxc++] = contrib;
  }
  for (int level = 0; level < nlevels; level++) {
    const int ul = K.T.ion_uniqueleveloffset[ui] + level;
    const double epsilon_current = K.T.level_epsilon[ul];
    const double nnlevel = popsT[(int64_t)ul * nne_cells];
    const double statweight = K.T.level_stat_weight[ul];
    const int nuptrans = K.T.level_nuptrans[ul];
    if (nuptrans > 0) {
      // the packed excitation terms (TeExcItem): one independent load per line instead of a dependent chain
      const TeExcItem *it = K.T.exc_items + K.T.level_uptrans_offset[ul];
#pragma unroll 2
      for (int ii = 0; ii < nuptrans; ii++) {
        const TeExcItem x = it[ii];
        const double C = nnlevel * te_col_exc(x, T_e, nne, statweight) * x.epsilon_trans;
        contrib += C;
      }
      cc[idxc++] = contrib;
    }
    if (i < (nions - 1) && level < ionisinglevels) {
      const int nt = K.T.level_nphixstargets[ul];
      for (int t = 0; t < nt; t++) {
        const int upper = get_phixsupperlevel(K, e, i, level, t);
        const double epsilon_upper = epsilon(K, e, i + 1, upper);
        const double epsilon_trans = epsilon_upper - epsilon_current;
        const double C = nnlevel * col_ionization_ratecoeff(K, T_e, nne, e, i, level, t, epsilon_trans) * epsilon_trans;
        contrib += C;
        cc[idxc++] = contrib;
      }
      for (int t = 0; t < nt; t++) {
        const double nnupperion = K.C.ionpop[(int64_t)k * ni + ui + 1];
        const double C = lut_interp(K, K.T.bfcooling_coeff, e, i, level, t, T_e) * nnupperion * nne;
        contrib += C;
        cc[idxc++] = contrib;
      }
    }
  }
}

// macroatom.cc:57-159 calculate_macroatom_transitionrates, one workitem per (cell, level) (ma_foreach_rate); with the
// macro-atom cache it also stores the running sums of the individual rates (cellhistory individ_* arrays).
// Workitems are ordered level-major (consecutive lanes = the same level in consecutive cells): every lane of
// a wave walks the same transition lists, so the atomic-data loads are wave-uniform and the loops do not
// diverge; only the cell's populations (level-major copy popsT) and temperatures differ per lane.
// With the cache, one launch covers levels [ul0, ul0 + nlev) and writes the exact double running sums
// position-major into the scratch S (S[(dbl_off(ul) - dbl_off(ul0)) * n_ne + pos * n_ne + k]: every store is 64
// consecutive doubles); k_mapack then turns them into the compact key records.  Scratch positions:
//   [9 totals | internal_down_same (nd) | internal_up_same (nu) | rad_deexc (nd) | rad_recomb (nr) |
//    internal_down_lower (nr) | internal_up_higher (nt)]     (each array in the reference's order)
// One launch covers the kn cells cells[0 .. kn): the cached cells (row order) with cache = true (scratch stride
// kn), the others with cache = false (totals into marates).
// k_marates' work for one (cell, level): the running sums into rec[p * stride] (cache), the action totals into pr
// (cache a template parameter: each instance's transition loop has one path, so the population loaded for the next
// transition is waited for without waiting for the running-sum stores issued after it)
template <bool cache>
DEVFN void marates_sums(const Ctx &K, int ul, int k, double t_mid, double *__restrict__ rec, int64_t stride,
                        double pr[ARTIS_MA_ACTION_COUNT]) {
  const int64_t nne_cells = K.C.n_nonempty;
  const int mgi = K.C.ne_mgi[k];
  const MaMeta mm = K.T.ma_meta[ul];
#define REC(p) rec[(int64_t)(p) * stride]
  const int cum_d = ARTIS_MA_ACTION_COUNT, cum_u = ARTIS_MA_ACTION_COUNT + mm.nd;
  const int cum_drad = ARTIS_MA_ACTION_COUNT + mm.nd + mm.nu, cum_rrad = cum_drad + mm.nd;
  const int cum_rint = cum_rrad + mm.nr, cum_uhi = cum_rint + mm.nr;
  for (int a = 0; a < ARTIS_MA_ACTION_COUNT; a++) pr[a] = 0.;
  const double *popsT = K.C.popsT + k;  // popsT[u * nne_cells]: level u of this lane's cell
#ifdef ARTIS_MARATES_PLAIN  // A/B: the plain ma_foreach_rate loop
  ma_foreach_rate(
#else
  ma_foreach_rate_pf(
#endif
      K, mgi, ul, t_mid, [&](int u) { return popsT[(int64_t)u * nne_cells]; },
      [&](int slot) { return K.C.corrphotT[(int64_t)slot * nne_cells + k]; },
      [&](int kind, int j, double R, double C, double et, double eg, double ec) {
        ma_accumulate(pr, kind, R, C, et, eg, ec);
#ifdef ARTIS_DIAG_MARATES_NOSTORE  // timing diagnostic only (the records are not written): the rates' compute alone
        if (false) {
#else
        if constexpr (cache) {
#endif
          if (kind == MA_KIND_DOWN) {
            REC(cum_drad + j) = pr[ARTIS_MA_ACTION_RADDEEXC];
            REC(cum_d + j) = pr[ARTIS_MA_ACTION_INTERNALDOWNSAME];
          } else if (kind == MA_KIND_RECOMB) {
            REC(cum_rrad + j) = pr[ARTIS_MA_ACTION_RADRECOMB];
            REC(cum_rint + j) = pr[ARTIS_MA_ACTION_INTERNALDOWNLOWER];
          } else if (kind == MA_KIND_UP) {
            REC(cum_u + j) = pr[ARTIS_MA_ACTION_INTERNALUPSAME];
          } else {
            REC(cum_uhi + j) = pr[ARTIS_MA_ACTION_INTERNALUPHIGHER];
          }
        }
        return false;
      });
  pr[ARTIS_MA_ACTION_INTERNALUPHIGHERNT] = ma_nt_total(K, mgi, ul);
  if constexpr (cache)
    for (int a = 0; a < ARTIS_MA_ACTION_COUNT; a++) REC(a) = pr[a];
#undef REC
}

// The rows of each level are padded to a multiple of 64 (MARATES_PAD), so that a wave never straddles two levels: the
// level index is then wave-uniform (readfirstlane), and the atomic data the rates read are scalar loads.
#define MARATES_PAD(kn) (((int64_t)(kn) + 63) & ~(int64_t)63)
template <bool cache>
__global__ void k_marates(Ctx K, int nts, int ul0, int nlev, double *__restrict__ S, const int32_t *__restrict__ cells,
                          int kn) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nl = K.T.nlevels_total;
  const int64_t knp = MARATES_PAD(kn);
  const int ul = __builtin_amdgcn_readfirstlane(ul0 + (int)(idx / knp));
  const int kr = (int)(idx % knp);
  if (ul >= ul0 + nlev || kr >= kn) return;
  const int k = cells[kr];
  // the scratch of level ul: 64-row groups, each [position][64 rows] (a wave's stores, and k_mapack's tile, are
  // contiguous runs of memory)
  const int64_t len = K.T.ma_dbl_off[ul + 1] - K.T.ma_dbl_off[ul];
  double *rec = cache ? S + (K.T.ma_dbl_off[ul] - K.T.ma_dbl_off[ul0]) * knp + (int64_t)(kr >> 6) * len * 64 + (kr & 63)
                      : nullptr;
  double pr[ARTIS_MA_ACTION_COUNT];
  marates_sums<cache>(K, ul, k, K.G.ts_mid[nts], rec, 64, pr);
  if constexpr (!cache) {
    double *out = K.C.marates + ((int64_t)k * nl + ul) * ARTIS_MA_ACTION_COUNT;
    for (int a = 0; a < ARTIS_MA_ACTION_COUNT; a++) out[a] = pr[a];
  }
}

// Exact running sums (scratch) -> the compact key records (engine_dev.h DevCells::ma_key): every sum divided by its
// action's total (the action totals by their grand total, summed in the reference's order, macroatom.cc:515-525) and
// rounded to 32 bits, split into halves.  One (level ul, 64 rows) tile, run by a block of 256 threads: 64 x 64
// (position x row) tiles through LDS, read along rows from the position-major scratch src (row stride n_s; rows
// c0 .. c0 + 63 of it, the first nvalid valid), written along positions (64 consecutive keys of one record per row:
// coalesced) into record rows row0 + c0 + j.
#ifndef MAPACK_P
#define MAPACK_P 64  // record positions per LDS tile (64: a wave stores whole 128-byte lines of a record row, 41 KB of
                     // LDS per block; 32: 24 KB, 6 blocks per CU, 7 % slower, profiles/r6y_precompute_ab.txt)
#endif
struct MapackLds {
  double tile[MAPACK_P][65];
  double norm[ARTIS_MA_ACTION_COUNT][64];  // action totals per row
  uint32_t akey[ARTIS_MA_ACTION_COUNT][64];
};
DEVFN void mapack_tile(const Ctx &K, int ul, const double *__restrict__ src, int64_t n_s, int64_t c0, int64_t nvalid,
                       int64_t row0, MapackLds &S) {
  constexpr int P = MAPACK_P, RS = 256 / MAPACK_P;  // positions per tile; rows a pass of the block covers
  const MaMeta mm = K.T.ma_meta[ul];
  const int len = ARTIS_MA_ACTION_COUNT + 2 * mm.nd + mm.nu + 2 * mm.nr + mm.nt;
  const MaLayout lay = ma_layout(mm.nd, mm.nu, mm.nr, mm.nt);
  const int tx = threadIdx.x % P, ty = threadIdx.x / P;
  // the tiles are double-buffered through registers: the next tile's loads are in flight while the current one is
  // converted and stored (the first one's with the action totals' loads)
  constexpr int NB = P * 64 / 256;  // doubles per thread and tile
  double buf[NB];
  auto fetch = [&](int p0) {
#pragma unroll
    for (int b = 0; b < NB; b++) {
      const int q = threadIdx.x + b * 256;  // (64 consecutive rows of one position per wave: coalesced)
      const int pp = q / 64, rr = q % 64;
      buf[b] = (p0 + pp < len && c0 + rr < nvalid) ? src[(int64_t)(p0 + pp) * n_s + c0 + rr] : 0.;
    }
  };
  fetch(0);
  __syncthreads();  // (the previous tile's readers of S are done)
  if (threadIdx.x < 64 && c0 + threadIdx.x < nvalid) {
    const int r = threadIdx.x;
    double pr[ARTIS_MA_ACTION_COUNT];
    double total = 0.;
    for (int a = 0; a < ARTIS_MA_ACTION_COUNT; a++) {
      pr[a] = src[(int64_t)a * n_s + c0 + r];
      S.norm[a][r] = pr[a];
      total += pr[a];
    }
    double rate = 0.;
    for (int a = 0; a < ARTIS_MA_ACTION_COUNT; a++) {
      rate += pr[a];
      S.akey[a][r] = ma_key32(rate, total);
    }
  }
  // segment boundaries of the record (positions >= 9): the action whose total normalises each
  const int b1 = ARTIS_MA_ACTION_COUNT + mm.nd, b2 = b1 + mm.nu, b3 = b2 + mm.nd, b4 = b3 + mm.nr, b5 = b4 + mm.nr;
  for (int p0 = 0; p0 < len; p0 += P) {
    __syncthreads();
#pragma unroll
    for (int b = 0; b < NB; b++) {
      const int q = threadIdx.x + b * 256;
      S.tile[q / 64][q % 64] = buf[b];
    }
    __syncthreads();
    if (p0 + P < len) fetch(p0 + P);
    const int p = p0 + tx;
    if (p < len) {
      const int a = (p < ARTIS_MA_ACTION_COUNT) ? -1
                    : (p < b1)                 ? ARTIS_MA_ACTION_INTERNALDOWNSAME
                    : (p < b2)                 ? ARTIS_MA_ACTION_INTERNALUPSAME
                    : (p < b3)                 ? ARTIS_MA_ACTION_RADDEEXC
                    : (p < b4)                 ? ARTIS_MA_ACTION_RADRECOMB
                    : (p < b5)                 ? ARTIS_MA_ACTION_INTERNALDOWNLOWER
                                               : ARTIS_MA_ACTION_INTERNALUPHIGHER;
      int sp;
      const int rp = ma_rec_pos(lay, p, mm.nd, mm.nu, &sp);
      // the rows of this position U at a time: their LDS terms and norms read together, then the keys (branch-free
      // ma_key32_nb) and stores -- one LDS round trip per U keys instead of two dependent ones per key
      constexpr int U = 4;
      static_assert(64 % (U * RS) == 0, "row groups of U");
      const int an = a < 0 ? 0 : a, pa = p < ARTIS_MA_ACTION_COUNT ? p : 0;
      for (int j0 = ty; j0 < 64; j0 += U * RS) {
        double v[U], nv[U];
        uint32_t ak[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
          const int j = j0 + u * RS;
          v[u] = S.tile[tx][j];
          nv[u] = S.norm[an][j];
          ak[u] = S.akey[pa][j];
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
          const int j = j0 + u * RS;
          if (c0 + j < nvalid) {
            const uint32_t key = (a < 0) ? ak[u] : ma_key32_nb(v[u], nv[u]);
            uint16_t *rec = K.C.ma_key + (row0 + c0 + j) * K.C.ma_key_stride + mm.rec_off;
            rec[rp] = (uint16_t)(key >> 16);
            rec[lay.hot + rp] = (uint16_t)(key & 0xffffu);
            if (sp >= 0) {  // also a block separator on the record's first line
              rec[sp] = (uint16_t)(key >> 16);
              rec[lay.hot + sp] = (uint16_t)(key & 0xffffu);
            }
          }
        }
      }
    }
  }
}

// one k_marates batch's scratch -> key records: block = (64-row group blockIdx.x, level ul0 + blockIdx.y).  (A
// grid-stride version, a few blocks per CU over the tiles, measured slower: 1.35 against 1.26 ms per batch.)
__global__ __launch_bounds__(256) void k_mapack(Ctx K, int ul0, const double *__restrict__ S) {
  __shared__ MapackLds L;
  const int ul = ul0 + blockIdx.y;
  const int64_t n_ne = K.C.ma_rows;  // the cached cells
  const int64_t g = blockIdx.x;
  const int64_t len = K.T.ma_dbl_off[ul + 1] - K.T.ma_dbl_off[ul];
  // (the level's scratch: 64-row groups [position][64 rows], k_marates)
  const double *src = S + (K.T.ma_dbl_off[ul] - K.T.ma_dbl_off[ul0]) * MARATES_PAD(n_ne) + g * len * 64;
  mapack_tile(K, ul, src, 64, 0, min((int64_t)64, n_ne - g * 64), g * 64, L);
}

// ---- level mode of the macro-atom key records (DevCells::ma_lptr): placement and build ----------------------
// A pair's value for the pool is its sampled jump count c per record line rl (a knapsack by density): bucket
// 1 + 2 floor(log2 v) + (the next bit of v) for v = 256 c / rl, half-octave steps; 0 for v == 0 with c > 0.
#define MA_LVL_NB 84
DEVFN int ma_lvl_bucket(uint32_t c, uint32_t rl) {
  const uint64_t v = ((uint64_t)c << 8) / rl;
  if (!v) return 0;
  const int e = 63 - __clzll((long long)v);
  const int half = e >= 1 ? (int)((v >> (e - 1)) & 1u) : 0;
  return 1 + 2 * e + half;
}
// k_lvl_buckets: over every (cell, level) pair's sampled jump count c since the last placement: [0] the jumps on
// pairs that had a record, [1] all jumps, [2 + b] the pool lines the pairs of density bucket b would take
__global__ __launch_bounds__(256) void k_lvl_buckets(Ctx K, const uint32_t *__restrict__ rec_lines,
                                                     unsigned long long *__restrict__ out, int64_t npairs) {
  __shared__ unsigned long long s[2 + MA_LVL_NB];
  for (int j = threadIdx.x; j < 2 + MA_LVL_NB; j += blockDim.x) s[j] = 0;
  __syncthreads();
  const int64_t nl = K.T.nlevels_total;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < npairs; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t c = K.C.ma_lhist[i];
    if (!c) continue;
    atomicAdd(&s[1], (unsigned long long)c);
    if (K.C.ma_lptr[i] != MA_NOLINE) atomicAdd(&s[0], (unsigned long long)c);
    const uint32_t rl = rec_lines[i % nl];
    if (rl) atomicAdd(&s[2 + ma_lvl_bucket(c, rl)], (unsigned long long)rl);
  }
  __syncthreads();
  for (int j = threadIdx.x; j < 2 + MA_LVL_NB; j += blockDim.x)
    if (s[j]) atomicAdd(&out[j], s[j]);
}

// after a placement: the counts decay by half (rounded up, so a pair walked once keeps its place at the end of the
// queue): pairs walked in earlier transports keep a claim on the pool, pairs walked often keep the front
__global__ __launch_bounds__(256) void k_lvl_decay(uint32_t *__restrict__ hist, int64_t npairs) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < npairs; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t c = hist[i];
    if (c) hist[i] = (c >> 1) + (c & 1u);
  }
}

#define MA_BUILD_MAX_DOUBLES 6144  // LDS terms of one level (48 KiB); a level with more never gets a record
// k_ma_build's LDS terms of a level (below).  The levels whose terms take at most 10 KiB are built by their own
// launch of that LDS size: 16 blocks per CU, 4 waves per SIMD with the kernel's 128 VGPRs (MA_BUILD_MINW), where
// sizing every block for the largest level of a large atom left 3 blocks per CU (round 6 until its last session: 20
// KiB and 169 VGPRs, 2 waves per SIMD)
#define MA_BUILD_SMALL 1280
static inline __host__ __device__ int64_t ma_build_doubles(const MaMeta &m) { return 3 * ((int64_t)m.nd + m.nr) + m.nu + m.nt; }
// k_lvl_select: the new DevCells::ma_lptr and the list of records to build.  have_hist == 0 (no transport yet):
// whole cells in nonempty-index order (centre outwards), pair (k, ul) at line k * row_lines + rl_off[ul] while it
// fits the pool.  Otherwise: density bucket above bt, or bucket bt while `rest` lines of it last.
// ctr: [0] pool lines taken, [1] records listed from the front (levels whose k_ma_build terms fit MA_BUILD_SMALL
// doubles of LDS), [2] lines taken from bucket bt, [3] records listed from the back (the larger levels)
__global__ __launch_bounds__(256) void k_lvl_select(Ctx K, const uint32_t *__restrict__ rec_lines,
                                                    const uint32_t *__restrict__ rl_off, uint32_t row_lines,
                                                    uint32_t *__restrict__ lptr, uint32_t *__restrict__ ctr,
                                                    int2 *__restrict__ list, int64_t list_cap, int64_t npairs, int bt,
                                                    uint32_t rest, uint64_t pool_lines, int have_hist,
                                                    int64_t small_max) {
  const int64_t nl = K.T.nlevels_total;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < npairs; i += (int64_t)gridDim.x * blockDim.x) {
    const int ul = (int)(i % nl), k = (int)(i / nl);
    const uint32_t rl = rec_lines[ul];
    uint32_t line = MA_NOLINE;
    if (rl && !have_hist) {
      const uint64_t l0 = (uint64_t)k * row_lines + rl_off[ul];
      if (l0 + rl <= pool_lines) {
        line = (uint32_t)l0;
        atomicAdd(&ctr[0], rl);
      }
    } else if (rl) {
      const uint32_t c = K.C.ma_lhist[i];
      if (c) {
        const int b = ma_lvl_bucket(c, rl);
        bool take = b > bt;
        if (b == bt) take = atomicAdd(&ctr[2], rl) + rl <= rest;
        if (take) line = atomicAdd(&ctr[0], rl);
      }
    }
    lptr[i] = line;
    if (line != MA_NOLINE) {
      const MaMeta mm = K.T.ma_meta[ul];
      if (ma_build_doubles(mm) <= small_max) {
        const uint32_t s = atomicAdd(&ctr[1], 1u);
        if (s < list_cap) list[s] = make_int2(k, ul);
      } else {
        const uint32_t s = atomicAdd(&ctr[3], 1u);
        if (s < list_cap) list[list_cap - 1 - s] = make_int2(k, ul);
      }
    }
  }
}

// k_ma_build: the key record of each listed (cell, level) pair, one wave per record -- what k_marates + k_mapack
// compute for a whole row, for one pair: the lanes evaluate the level's individual rates (ma_rate_at) and stage
// the terms of its eight action sums in LDS; eight lanes then add up one action each in the reference's list order
// (macroatom.cc:57-159: every action's running sum only involves its own terms, so the chains are independent and
// equal to ma_accumulate's sequence bit for bit); the lanes write the normalised 32-bit keys at their record
// positions (ma_rec_pos, with the block separators).
#ifndef MA_BUILD_MINW
#define MA_BUILD_MINW 4  // waves per SIMD k_ma_build is compiled for (128 VGPRs; with the small launch's 10 KiB of LDS, 4
                         // waves per SIMD: level-mode precompute 1.69 -> 1.34 s, profiles/r6u_level_mode_ab.txt)
#endif
__global__ __launch_bounds__(64, MA_BUILD_MINW) void k_ma_build(Ctx K, const int2 *__restrict__ list, uint32_t nlist,
                                                              int nts) {
  extern __shared__ double sb[];
  const int lane = threadIdx.x;
  const int64_t nl = K.T.nlevels_total;
  const double t_mid = K.G.ts_mid[nts];
  for (uint32_t e = blockIdx.x; e < nlist; e += gridDim.x) {
    const int2 kl = list[e];
    const int k = kl.x, ul = kl.y;
    const int mgi = K.C.ne_mgi[k];
    const MaMeta mm = K.T.ma_meta[ul];
    const int nd = mm.nd, nr = mm.nr, nu = mm.nu, nt = mm.nt;
    double *Drad = sb, *Dcol = Drad + nd, *Dsame = Dcol + nd, *Rint = Dsame + nd, *Rrad = Rint + nr,
           *Rcol = Rrad + nr, *Usame = Rcol + nr, *Uhi = Usame + nu;
    const double ec = K.T.level_epsilon[ul];
    const double *pops = K.C.pops + (int64_t)k * nl;
    const double *corr = K.C.corrphot + (int64_t)k * K.T.ntargets_total;
    auto pop = [&](int u) { return pops[u]; };
    auto cph = [&](int s) { return corr[s]; };
    __syncthreads();  // the previous record's LDS reads are done
    for (int pos = lane; pos < nd + nr + nu + nt; pos += 64) {
      const MaItem it = ma_rate_at(K, mgi, ul, t_mid, pos, pop, cph);
      if (it.kind == MA_KIND_DOWN) {
        Drad[it.j] = it.R * it.et;
        Dcol[it.j] = it.C * it.et;
        Dsame[it.j] = (it.R + it.C) * it.eg;
      } else if (it.kind == MA_KIND_RECOMB) {
        Rint[it.j] = (it.R + it.C) * it.eg;
        Rrad[it.j] = it.R * it.et;
        Rcol[it.j] = it.C * it.et;
      } else if (it.kind == MA_KIND_UP) {
        Usame[it.j] = (it.R + it.C + 0.) * ec;
      } else {
        Uhi[it.j] = (it.R + it.C) * ec;
      }
    }
    __syncthreads();
    if (lane < 8) {  // one running sum per lane, in list order, in place
      double *a = lane == 0 ? Drad : lane == 1 ? Dcol : lane == 2 ? Dsame : lane == 3 ? Rint : lane == 4 ? Rrad
                  : lane == 5 ? Rcol : lane == 6 ? Usame : Uhi;
      const int len = lane < 3 ? nd : lane < 6 ? nr : lane == 6 ? nu : nt;
      // (eight terms read at a time, then added one after another and written back: one LDS round trip per eight
      // additions instead of one per addition -- the same sums in the same order)
      double r = 0.;
      int j = 0;
      for (; j + 8 <= len; j += 8) {
        double x[8];
#pragma unroll
        for (int q = 0; q < 8; q++) x[q] = a[j + q];
#pragma unroll
        for (int q = 0; q < 8; q++) {
          r += x[q];
          x[q] = r;
        }
#pragma unroll
        for (int q = 0; q < 8; q++) a[j + q] = x[q];
      }
      for (; j < len; j++) {
        r += a[j];
        a[j] = r;
      }
    }
    __syncthreads();
    double pr[ARTIS_MA_ACTION_COUNT];
    pr[ARTIS_MA_ACTION_RADDEEXC] = nd ? Drad[nd - 1] : 0.;
    pr[ARTIS_MA_ACTION_COLDEEXC] = nd ? Dcol[nd - 1] : 0.;
    pr[ARTIS_MA_ACTION_INTERNALDOWNSAME] = nd ? Dsame[nd - 1] : 0.;
    pr[ARTIS_MA_ACTION_INTERNALDOWNLOWER] = nr ? Rint[nr - 1] : 0.;
    pr[ARTIS_MA_ACTION_RADRECOMB] = nr ? Rrad[nr - 1] : 0.;
    pr[ARTIS_MA_ACTION_COLRECOMB] = nr ? Rcol[nr - 1] : 0.;
    pr[ARTIS_MA_ACTION_INTERNALUPSAME] = nu ? Usame[nu - 1] : 0.;
    pr[ARTIS_MA_ACTION_INTERNALUPHIGHER] = nt ? Uhi[nt - 1] : 0.;
    pr[ARTIS_MA_ACTION_INTERNALUPHIGHERNT] = ma_nt_total(K, mgi, ul);
    double total = 0.;
    for (int a = 0; a < ARTIS_MA_ACTION_COUNT; a++) total += pr[a];
    const MaLayout lay = ma_layout(nd, nu, nr, nt);
    uint16_t *rec = K.C.ma_key + (size_t)K.C.ma_lptr[(int64_t)k * nl + ul] * 64;
    // positions in k_marates' scratch order: [9 totals | down-same nd | up-same nu | rad_deexc nd | rad_recomb nr |
    // internal_down_lower nr | internal_up_higher nt]
    const int len = ARTIS_MA_ACTION_COUNT + 2 * nd + nu + 2 * nr + nt;
    for (int p = lane; p < len; p += 64) {
      uint32_t key;
      if (p < ARTIS_MA_ACTION_COUNT) {
        double rate = 0.;
        for (int a = 0; a <= p; a++) rate += pr[a];
        key = ma_key32(rate, total);
      } else {
        int q = p - ARTIS_MA_ACTION_COUNT;
        if (q < nd) {
          key = ma_key32(Dsame[q], pr[ARTIS_MA_ACTION_INTERNALDOWNSAME]);
        } else if ((q -= nd) < nu) {
          key = ma_key32(Usame[q], pr[ARTIS_MA_ACTION_INTERNALUPSAME]);
        } else if ((q -= nu) < nd) {
          key = ma_key32(Drad[q], pr[ARTIS_MA_ACTION_RADDEEXC]);
        } else if ((q -= nd) < nr) {
          key = ma_key32(Rrad[q], pr[ARTIS_MA_ACTION_RADRECOMB]);
        } else if ((q -= nr) < nr) {
          key = ma_key32(Rint[q], pr[ARTIS_MA_ACTION_INTERNALDOWNLOWER]);
        } else {
          key = ma_key32(Uhi[q - nr], pr[ARTIS_MA_ACTION_INTERNALUPHIGHER]);
        }
      }
      int sp;
      const int rp = ma_rec_pos(lay, p, nd, nu, &sp);
      rec[rp] = (uint16_t)(key >> 16);
      if (!K.C.ma_hi_only) rec[lay.hot + rp] = (uint16_t)(key & 0xffffu);
      if (sp >= 0) {
        rec[sp] = (uint16_t)(key >> 16);
        if (!K.C.ma_hi_only) rec[lay.hot + sp] = (uint16_t)(key & 0xffffu);
      }
    }
  }
}

// DevCells::linecoef: the Sobolev coefficient (B_lu n_l - B_ul n_u) * HCLIGHTOVERFOURPI of every line in every
// non-empty cell, in get_event's operation order (rpkt.cc:168-187); lanes run along a cell's row (coalesced
// writes, line records from L2, population gathers from the cell's 29 kB row).  A block takes 256 lines of
// LINECOEF_R consecutive rows: the line record is loaded once, and the rows' population gathers are all in flight
// before the stores (one row per block and thread: the launch was bound by dispatching 12.8 M short blocks).
#ifndef LINECOEF_R
#define LINECOEF_R 8
#endif
__global__ __launch_bounds__(256) void k_linecoef(Ctx K) {
  const int64_t li = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (li >= K.C.linecoef_stride) return;
  const bool in = li < K.T.nlines;
  LineTau r{};
  if (in) r = K.T.line_tau[li];
  bool neg = false;
  for (int k0 = blockIdx.y * LINECOEF_R; k0 < K.C.linecoef_rows; k0 += gridDim.y * LINECOEF_R) {
    double v[LINECOEF_R];
#pragma unroll
    for (int q = 0; q < LINECOEF_R; q++) {
      v[q] = 0.;
      if (in && k0 + q < K.C.linecoef_rows) {
        const double *pops = K.C.pops + (int64_t)(k0 + q) * K.T.nlevels_total;
        const double n_u = pops[r.ul_upper], n_l = pops[r.ul_lower];
        v[q] = (r.B_lu * n_l - r.B_ul * n_u) * ARTIS_HCLIGHTOVERFOURPI;
        neg = neg || v[q] < 0.;
      }
    }
#pragma unroll
    for (int q = 0; q < LINECOEF_R; q++)
      if (k0 + q < K.C.linecoef_rows) K.C.linecoef[(int64_t)(k0 + q) * K.C.linecoef_stride + li] = v[q];
  }
  // (one atomic per wave until the flag is seen set: an atomic per wave on one address serialises the launch)
  if (__any(neg) && __lane_id() == 0 && !*(volatile int32_t *)K.C.linecoef_neg) atomicOr(K.C.linecoef_neg, 1);
}

// k_linecoef with the populations in LDS: a block copies LINECOEF_LDS_R consecutive rows of populations (contiguous
// in DevCells::pops) into LDS once and walks every line for them, the line records from L2.  The gathers of the
// kernel above -- two per line and row, ~60 distinct cache lines per wave instruction -- bound it at the vector
// memory pipeline (27 ms per upload of the bench model for a 49 GB table); from LDS they cost a few cycles, and the
// kernel is left with its stores.  The same expression, so the same table bit for bit.  nr_max rows fit the
// LINECOEF_LDS_DOUBLES of LDS (host: models whose levels do not fit one row take the kernel above).
#define LINECOEF_LDS_DOUBLES 18432  // 144 KiB: 5 rows of the bench's 3 603 levels
__global__ __launch_bounds__(1024) void k_linecoef_lds(Ctx K, int nr_max) {
  __shared__ double sp[LINECOEF_LDS_DOUBLES];
  const int64_t nl = K.T.nlevels_total, rows = K.C.linecoef_rows, stride = K.C.linecoef_stride;
  const int nlines = K.T.nlines;
  bool neg = false;
  for (int64_t k0 = (int64_t)blockIdx.x * nr_max; k0 < rows; k0 += (int64_t)gridDim.x * nr_max) {
    const int nr = (int)min((int64_t)nr_max, rows - k0);
    __syncthreads();  // (the previous rows' readers are done)
    const double *src = K.C.pops + k0 * nl;
    for (int64_t q = threadIdx.x; q < nr * nl; q += blockDim.x) sp[q] = src[q];
    __syncthreads();
    for (int64_t li = threadIdx.x; li < stride; li += blockDim.x) {
      const bool in = li < nlines;
      LineTau r{};
      if (in) r = K.T.line_tau[li];
      double *out = K.C.linecoef + k0 * stride + li;
      for (int q = 0; q < nr; q++) {
        double v = 0.;
        if (in) {
          const double n_u = sp[q * nl + r.ul_upper], n_l = sp[q * nl + r.ul_lower];
          v = (r.B_lu * n_l - r.B_ul * n_u) * ARTIS_HCLIGHTOVERFOURPI;
          neg = neg || v < 0.;
        }
        out[q * stride] = v;
      }
    }
  }
  if (__any(neg) && __lane_id() == 0 && !*(volatile int32_t *)K.C.linecoef_neg) atomicOr(K.C.linecoef_neg, 1);
}

// out[c * rows + r] = in[r * cols + c], through a 64x64 LDS tile (one wave reads rows, writes columns)
__global__ __launch_bounds__(256) void k_transpose(const double *__restrict__ in, double *__restrict__ out,
                                                   int64_t rows, int64_t cols) {
  __shared__ double tile[64][65];
  const int64_t r0 = (int64_t)blockIdx.y * 64, c0 = (int64_t)blockIdx.x * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int j = ty; j < 64; j += 4) {
    const int64_t r = r0 + j, c = c0 + tx;
    if (r < rows && c < cols) tile[j][tx] = in[r * cols + c];
  }
  __syncthreads();
  for (int j = ty; j < 64; j += 4) {
    const int64_t c = c0 + j, r = r0 + tx;
    if (r < rows && c < cols) out[c * rows + r] = tile[tx][j];
  }
}

// The drop-in boundary's packet array (AoS, 304-byte records) <-> the packet store (packet_soa.h groups), 64 packets
// per block through LDS: the block's 19 kB of records are read (or written) as one contiguous run, and each group's
// words as contiguous runs of that group (one packet per thread touched 38 records' lines once per word: the
// transpose fetched 15x the array, profiles/pmc_r5x_bench.json).  Slot -> word maps of the groups:
__constant__ int8_t c_hot_word[16] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 18, 33};
__constant__ int8_t c_cold_word[20] = {19, 21, 22, 23, 24, 36, 37, 20, 14, 15, 16, 17, 25, 26, 27, 28, 29, 30, 32, 35};
__constant__ int8_t c_rest_word[2] = {31, 34};
constexpr int8_t h_hot_word[16] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 18, 33};
constexpr int8_t h_cold_word[20] = {19, 21, 22, 23, 24, 36, 37, 20, 14, 15, 16, 17, 25, 26, 27, 28, 29, 30, 32, 35};
constexpr int8_t h_rest_word[2] = {31, 34};
constexpr bool pkt_maps_ok() {
  for (int s = 0; s < 16; s++)
    if (pkt_word_group(h_hot_word[s]) != 0 || pkt_word_slot(h_hot_word[s]) != s) return false;
  for (int s = 0; s < 20; s++)
    if (pkt_word_group(h_cold_word[s]) != 1 || pkt_word_slot(h_cold_word[s]) != s) return false;
  for (int s = 0; s < 2; s++)
    if (pkt_word_group(h_rest_word[s]) != 2 || pkt_word_slot(h_rest_word[s]) != s) return false;
  return 16 + 20 + 2 == PKT_WORDS;
}
static_assert(pkt_maps_ok(), "slot -> word maps agree with packet_soa.h");
#define XPOSE_PKTS 64
__global__ __launch_bounds__(256) void k_aos_to_soa(const uint64_t *__restrict__ aos, uint64_t *__restrict__ soa,
                                                    int64_t n) {
  __shared__ uint64_t s[XPOSE_PKTS * PKT_WORDS];
  const int64_t p0 = (int64_t)blockIdx.x * XPOSE_PKTS;
  const int np = (int)min((int64_t)XPOSE_PKTS, n - p0);
  for (int q = threadIdx.x; q < np * PKT_WORDS; q += blockDim.x) s[q] = aos[p0 * PKT_WORDS + q];
  __syncthreads();
  for (int q = threadIdx.x; q < np * 16; q += blockDim.x)
    soa[p0 * 16 + q] = s[(q >> 4) * PKT_WORDS + c_hot_word[q & 15]];
  for (int q = threadIdx.x; q < np * 20; q += blockDim.x) {
    const int p = q / 20, sl = q % 20;
    soa[16 * n + (p0 + p) * PKT_COLD_WIDTH + sl] = s[p * PKT_WORDS + c_cold_word[sl]];
  }
  for (int q = threadIdx.x; q < np * 2; q += blockDim.x)
    soa[(16 + PKT_COLD_WIDTH) * n + p0 * 2 + q] = s[(q >> 1) * PKT_WORDS + c_rest_word[q & 1]];
}
__global__ __launch_bounds__(256) void k_soa_to_aos(const uint64_t *__restrict__ soa, uint64_t *__restrict__ aos,
                                                    int64_t n) {
  __shared__ uint64_t s[XPOSE_PKTS * PKT_WORDS];
  const int64_t p0 = (int64_t)blockIdx.x * XPOSE_PKTS;
  const int np = (int)min((int64_t)XPOSE_PKTS, n - p0);
  for (int q = threadIdx.x; q < np * 16; q += blockDim.x)
    s[(q >> 4) * PKT_WORDS + c_hot_word[q & 15]] = soa[p0 * 16 + q];
  for (int q = threadIdx.x; q < np * 20; q += blockDim.x) {
    const int p = q / 20, sl = q % 20;
    s[p * PKT_WORDS + c_cold_word[sl]] = soa[16 * n + (p0 + p) * PKT_COLD_WIDTH + sl];
  }
  for (int q = threadIdx.x; q < np * 2; q += blockDim.x)
    s[(q >> 1) * PKT_WORDS + c_rest_word[q & 1]] = soa[(16 + PKT_COLD_WIDTH) * n + p0 * 2 + q];
  __syncthreads();
  for (int q = threadIdx.x; q < np * PKT_WORDS; q += blockDim.x) aos[p0 * PKT_WORDS + q] = s[q];
}

// update_packets.cc:234-333 (pass loop flattened, deviation D5) + do_packet update_packets.cc:137-202
#define TRANSPORT_BLOCK 256
__global__ __launch_bounds__(TRANSPORT_BLOCK) void k_transport(const Ctx *__restrict__ ctxp, uint64_t *__restrict__ soa, int64_t n, int nts,
                                                              double t2) {
  CTX_IN_LDS(ctxp)
  __shared__ unsigned long long s_ctr[ARTIS_COUNTER_COUNT + 1];
  __shared__ unsigned long long s_work[ARTIS_WORK_COUNT];
  __shared__ double s_cmflum[TRANSPORT_BLOCK / 64];
  for (int j = threadIdx.x; j < ARTIS_COUNTER_COUNT + 1; j += blockDim.x) s_ctr[j] = 0;
  for (int j = threadIdx.x; j < ARTIS_WORK_COUNT; j += blockDim.x) s_work[j] = 0;
  __syncthreads();
  LocalCounters L;
  L.ctr = &s_ctr[0];
  L.work = &s_work[0];
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  double cmf_lum = 0.;
  if (i < n) {
    Pkt p;
    pkt_load(soa, n, i, p);
    p.interactions = 0;  // update_packets.cc:285-288
    p.scat_count = 0;
    if (p.type != ARTIS_TYPE_ESCAPE && p.prop_time < t2) {
      lwork(L, WK_PACKETS_ACTIVE, 1);
      Tx x(K, L);
      x.nts = nts;
      x.rng = artis_rng_init(K.R.seed, p.number, nts, K.R.rank);
      long long iters = 0;
      while (x.ok && p.type != ARTIS_TYPE_ESCAPE && p.prop_time < t2) {
        if (++iters > 2000000ll) {
          x.err(ERR_STUCK, p.number, 0);
          break;
        }
        const int pkt_type = p.type;
        if (pkt_type == ARTIS_TYPE_RPKT) {
          while (x.ok && do_rpkt_step(x, p, t2)) {
          }
          if (p.type == ARTIS_TYPE_ESCAPE) {
            cmf_lum += p.e_cmf;
            lwork(L, WK_ESCAPED, 1);
          }
        } else if (pkt_type == ARTIS_TYPE_KPKT || pkt_type == ARTIS_TYPE_PRE_KPKT) {
          const int mgi = cell_mgi(K, p.where);
          if (pkt_type == ARTIS_TYPE_PRE_KPKT || K.C.thick[mgi] == 1)
            do_kpkt_bb(x, p);
          else
            do_kpkt(x, p, t2);
        } else if (pkt_type == ARTIS_TYPE_MA) {
          do_macroatom(x, p);
        } else if (is_gamma_family(pkt_type) && K.T.g_nlines) {
          PelletInfo pi;
          pellet_info_load(soa, n, i, pi);
          do_gamma_family_step(x, p, pi, t2);
        } else {
          x.err(ERR_UNSUPPORTED_TYPE, p.number, pkt_type);
        }
      }
    }
    pkt_store(soa, n, i, p);
  }
  // cmf_lum: wave reduction then one atomic per block (update_packets.cc:161)
  for (int off = 32; off > 0; off >>= 1) cmf_lum += __shfl_down(cmf_lum, off, 64);
  if ((threadIdx.x & 63) == 0) s_cmflum[threadIdx.x >> 6] = cmf_lum;
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0.;
    for (int w = 0; w < TRANSPORT_BLOCK / 64; w++) s += s_cmflum[w];
    if (s != 0.) unsafeAtomicAdd(&K.E.scalars[0], s);
  }
  for (int j = threadIdx.x; j < ARTIS_COUNTER_COUNT + 1; j += blockDim.x)
    if (s_ctr[j]) atomicAdd(&K.E.counters[j], s_ctr[j]);
  for (int j = threadIdx.x; j < ARTIS_WORK_COUNT; j += blockDim.x)
    if (s_work[j]) atomicAdd(&K.E.work[j], s_work[j]);
}

// pack estimators into one double block (for an RCCL all-reduce by the caller) and back
__global__ void k_pack_counts(const int32_t *ecounter, const int32_t *acounter, const unsigned long long *counters,
                              double *dst, int nlines, int dir) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n = 2 * (int64_t)nlines + ARTIS_COUNTER_COUNT + 1;
  if (i >= n) return;
  if (dir == 0) {
    if (i < nlines)
      dst[i] = ecounter[i];
    else if (i < 2 * nlines)
      dst[i] = acounter[i - nlines];
    else
      dst[i] = (double)counters[i - 2 * nlines];
  } else {
    if (i < nlines)
      const_cast<int32_t *>(ecounter)[i] = (int32_t)llrint(dst[i]);
    else if (i < 2 * nlines)
      const_cast<int32_t *>(acounter)[i - nlines] = (int32_t)llrint(dst[i]);
    else
      const_cast<unsigned long long *>(counters)[i - 2 * nlines] = (unsigned long long)llrint(dst[i]);
  }
}

// ================================================================================================= host side
namespace {

struct Engine {
  bool initialised = false;
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr, ev2 = nullptr;
  std::vector<void *> allocs;
  Ctx K{};
  artis_run_params params{};
  // sizes
  int npts_model = 0, nelements = 0, maxnions = 0, nions_total = 0, nlines = 0, ngrid = 0, ntstep = 0;
  int64_t n_est_doubles = 0;  // J..bfheat + scalars
  int64_t ma_key_stride = 0;          // 16-bit keys per cell block of the macro-atom cache
  bool ma_cache_ok = true;             // the atomic data fit the cache's record layout (engine_dev.h ma_layout)
  std::vector<int64_t> h_dbl_off;     // per level: offset (doubles) of its exact sums in the k_marates scratch
  double *d_marec_scratch = nullptr;  // k_marates output, [position][cell] per level (k_mapack input)
  // macro-atom key records (DevCells::ma_row / ma_bin): row of each cell (row mode), the cell of each bin
  int32_t *d_ma_row = nullptr, *d_ma_bin = nullptr, *d_ma_bincell = nullptr;
  // level mode (DevCells::ma_lptr): pool capacity, record size per level in 128-byte lines (0: never recorded),
  // the activity histogram of the walks since the last placement, and the placement's bookkeeping
  uint32_t *d_ma_lptr = nullptr, *d_ma_lhist = nullptr, *d_lvl_ctr = nullptr;
  const uint32_t *d_rec_lines = nullptr, *d_rl_off = nullptr;
  uint32_t row_lines = 0;  // pool lines of one whole cell's records (the initial placement)
  unsigned long long *d_lvl_buckets = nullptr;
  int2 *d_build_list = nullptr;
  int64_t build_list_cap = 0;
  int64_t ma_level_small = 0, ma_level_large = 0;  // the build list's front (small levels) and back (large) parts
  uint64_t ma_pool_lines = 0;
  std::vector<uint32_t> h_rec_lines;
  int64_t ma_build_lds_doubles = 0;
  bool ma_lhist_ready = false;
  bool ma_initial_placement = false;  // the current placement had no activity to go by (whole cells)
  int64_t ma_level_records = 0, ma_level_lines = 0;  // records / pool lines of the current placement
  // level mode: sampled jumps on pairs that had a record / on all pairs, over the transports before the last placement
  int64_t ma_acts_cached = 0, ma_acts_total = 0;
  int64_t marec_scratch_doubles = 0;
  double *d_estblock = nullptr;
  int32_t *d_target_ul = nullptr, *d_target_t = nullptr;
  bool have_cells = false;
  int cellstate_nts = -1;
  int cap_nonempty = 0;
  // cell-state device buffers
  float *d_cellf = nullptr;  // packed float arrays
  int16_t *d_thick = nullptr;
  float *d_abund = nullptr, *d_glp = nullptr, *d_pf = nullptr;
  double *d_totcool = nullptr, *d_ccion = nullptr, *d_renorm = nullptr;
  // nebular inputs (device copies, npts_model-indexed) and the NO_LUT integration workspace
  double *d_nltepops = nullptr, *d_ntdep = nullptr, *d_ntY = nullptr;
  float *d_rfTR = nullptr, *d_rfW = nullptr, *d_bfest = nullptr, *d_ntprob = nullptr, *d_ntionen = nullptr;
  QagWs qag{};
  int32_t *d_bfcol = nullptr;  // bflist index -> element * maxnions + ion (spectra emission columns)
  int qag_waves = 0;
  int64_t nbf_est = 0, nbins_est = 0;  // nebular estimator sections of the block (0 when off)
  int32_t *d_ne_index = nullptr, *d_ne_mgi = nullptr;
  // packets
  uint64_t *d_soa = nullptr, *d_aos = nullptr, *d_snapshot = nullptr;
  int64_t cap_pkts = 0, npkts = 0;
  bool have_snapshot = false;
  // wavefront engine (wavefront.h)
  WaveState W{};
  uint32_t *h_ctr = nullptr;  // pinned [2][NQUEUES * 2]
  hipEvent_t ev_round[2] = {nullptr, nullptr};
  int wave_grid = 2048;
  bool use_megakernel = false;
  bool ma_level_coop = false;  // level mode: k_ma makes the jumps without a record itself (else k_ma_exact)
  Ctx *d_ctx = nullptr;           // device copy of K for the transport kernels
  int ma_occ = 1;                 // k_ma minimum waves per SIMD (launch bounds): 1 or 8
  uint32_t *d_binoffs = nullptr;  // exclusive prefix sums of W.bins
  void *d_scan_tmp = nullptr;
  size_t scan_tmp_bytes = 0;
  int64_t last_rounds = 0;
  // per kernel class (rpkt, ma, kpkt, classify+bookkeeping): summed device time and launch count of the last
  // transport, from events bracketing every launch
  std::vector<hipEvent_t> tev;
  std::vector<int> tev_class;
  size_t tev_used = 0;
  double last_kernel_ms[ARTIS_KCLASS_COUNT] = {0};
  int64_t last_kernel_launches[ARTIS_KCLASS_COUNT] = {0};
  double last_transport_ms = 0., last_precompute_ms = 0.;
  int64_t last_work[ARTIS_WORK_COUNT] = {0};
  // virtual packets (vpkt.h): device accumulators and the spawn buffer (sized per update)
  int64_t vpkt_cap_param = 0;
  std::vector<int32_t> h_anumber;  // artis_atomic_tables.elem_anumber
  std::vector<double> h_ion_ionpot;  // artis_atomic_tables.ion_ionpot (get_mean_binding_energy)
  double last_nlte_ms = 0.;
  std::vector<int32_t> h_line_elem;  // artis_atomic_tables.line_elementindex (virtual-packet line masks)
  double *d_vpkt_spawn = nullptr;
  uint32_t vpkt_spawn_cap = 0;
  uint32_t *d_qsnap = nullptr;    // queue count when the current k_rpkt / k_kpkt launch started (vpkt_drain)
  // spawn sort (DevVpkt::perm): keys / indices in and out, hipcub temp storage, sized for vpkt_spawn_cap
  uint32_t *d_vkey = nullptr, *d_vkey2 = nullptr, *d_vidx = nullptr, *d_vperm = nullptr;
  void *d_vsort_tmp = nullptr;
  size_t vsort_tmp_bytes = 0;
  uint32_t *h_vcount = nullptr;   // pinned: spawn count before a flush
  bool vpkt_sort = true;          // ARTIS_VPKT_SORT=0: trace in buffer order
  uint32_t *h_vfull = nullptr;    // pinned: DevVpkt::full after a launch
  int64_t vpkt_drains = 0;        // launches resumed after a full spawn buffer (last update_packets)
  bool r_binned = false;          // bin the R queue by cell before k_rpkt (ARTIS_GPU_R_BIN=1)
  bool ma_bin_blk = true;         // few cells: block-local M-queue binning (ARTIS_GPU_MA_BIN_BLK=0: per-entry atomics)
  bool ma_pre_on = true;          // M-queue pre-tickets (WaveState::ma_pre; ARTIS_GPU_MA_PRE=0: gathered by the scatter)
  bool mf_rec_on = true;          // F-queue records (WaveState::mf_rec; ARTIS_GPU_MF_REC=0: the per-packet pend arrays)
  bool bin_push_on = true;        // M queue binned by its producers (WaveState::bin_push; ARTIS_GPU_BIN_PUSH=0: k_ma_bin)
  int rpkt_walk = -1;             // k_rpkt's bounded line walk: -1 by the previous transport's lines per step, 0 off, 1 on
  bool rpkt_coop = true;          // detailed-bf models: wave-made continuum sums in k_rpkt (ARTIS_GPU_RPKT_COOP=0: per lane)
  std::vector<hipEvent_t> vev;  // (start, end) pairs around the k_vpkt launches of the last update
  size_t vev_used = 0;
  double last_vpkt_ms = 0.;
  int64_t last_vpkt_work[4] = {0, 0, 0, 0};
  int64_t last_vpkt_spawns = 0, last_vpkt_traces = 0;
  // RCCL communicator of this rank (artis_gpu_comm_init) and the packed block it all-reduces
  ncclComm_t comm = nullptr;
  int comm_ranks = 0;
  double *d_redblock = nullptr;
  double last_te_ms = 0.;
  std::string last_error;
};
Engine G;

#define HIPCHK(x)                                                                             \
  do {                                                                                        \
    hipError_t e_ = (x);                                                                      \
    if (e_ != hipSuccess) {                                                                   \
      G.last_error = std::string(#x) + ": " + hipGetErrorString(e_);                          \
      return ARTIS_ERR_HIP;                                                                   \
    }                                                                                         \
  } while (0)

template <typename T>
int dalloc(T **p, size_t count) {
  if (count == 0) count = 1;
  HIPCHK(hipMalloc((void **)p, count * sizeof(T)));
  G.allocs.push_back((void *)*p);
  return 0;
}
template <typename T>
int dupload(const T **dst, const T *src, size_t count) {
  T *d = nullptr;
  if (dalloc(&d, count)) return ARTIS_ERR_HIP;
  if (count && src) HIPCHK(hipMemcpy(d, src, count * sizeof(T), hipMemcpyHostToDevice));
  *dst = d;
  return 0;
}

// The M-queue bins (DevCells::ma_bin, the cell of each bin ma_bincell) in `order`, and in row mode cell k's
// records at row k.  Placement never changes a result.
int ma_place(const std::vector<int32_t> &order) {
  const int n = G.K.C.n_nonempty;
  std::vector<int32_t> row(n, -1), bin(n);
  for (int b = 0; b < n; b++) {
    const int k = order[b];
    if (G.K.C.ma_rows > 0) row[k] = k;
    bin[k] = b;
  }
  HIPCHK(hipMemcpy(G.d_ma_row, row.data(), n * sizeof(int32_t), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(G.d_ma_bin, bin.data(), n * sizeof(int32_t), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(G.d_ma_bincell, order.data(), n * sizeof(int32_t), hipMemcpyHostToDevice));
  return 0;
}

// the small-level threshold of the build list (ARTIS_GPU_MA_BUILD_SMALL doubles overrides MA_BUILD_SMALL: tests run
// both launches on small atoms)
int64_t ma_build_small() {
  const char *e = getenv("ARTIS_GPU_MA_BUILD_SMALL");
  return e ? std::max<int64_t>(0, atoll(e)) : (int64_t)MA_BUILD_SMALL;
}

// Level mode, every artis_gpu_upload_cellstate: which (cell, level) pairs get a key record (DevCells::ma_lptr) and
// the list k_ma_build fills.  Before any transport: whole cells, centre outwards, while the pool lasts.  After:
// the pairs with the most (sampled) jumps since the last placement -- a threshold on log2 of the count found from
// the pool lines per count bucket, the pairs of the threshold bucket while the rest of the pool lasts.
int ma_level_place() {
  const int64_t npairs = (int64_t)G.K.C.n_nonempty * G.K.T.nlevels_total;
  const unsigned B = 256, nb = (unsigned)std::min<int64_t>((npairs + B - 1) / B, 1 << 20);
  HIPCHK(hipMemsetAsync(G.d_lvl_ctr, 0, 4 * sizeof(uint32_t), G.stream));
  int bt = MA_LVL_NB;  // threshold bucket (none -- the initial placement)
  uint64_t rest = 0;
  if (G.ma_lhist_ready) {
    HIPCHK(hipMemsetAsync(G.d_lvl_buckets, 0, (2 + MA_LVL_NB) * sizeof(unsigned long long), G.stream));
    k_lvl_buckets<<<nb, B, 0, G.stream>>>(G.K, G.d_rec_lines, G.d_lvl_buckets, npairs);
    unsigned long long h[2 + MA_LVL_NB];
    HIPCHK(hipMemcpyAsync(h, G.d_lvl_buckets, sizeof h, hipMemcpyDeviceToHost, G.stream));
    HIPCHK(hipStreamSynchronize(G.stream));
    // h[0]: sampled jumps on pairs with a record, h[1]: all, h[2 + b]: pool lines wanted per density bucket b
    if (h[1] == 0) return 0;  // no walk since the last placement: keep it (its list rebuilds the records)
    uint64_t cum = 0;
    bt = -1;  // (everything fits)
    for (int b = MA_LVL_NB - 1; b >= 0; b--) {
      if (cum + h[2 + b] > G.ma_pool_lines) {
        bt = b;
        break;
      }
      cum += h[2 + b];
    }
    rest = G.ma_pool_lines - cum;
  }
  k_lvl_select<<<nb, B, 0, G.stream>>>(G.K, G.d_rec_lines, G.d_rl_off, G.row_lines, G.d_ma_lptr, G.d_lvl_ctr,
                                       G.d_build_list, G.build_list_cap, npairs, bt,
                                       (uint32_t)std::min<uint64_t>(rest, 0xffffffffu), G.ma_pool_lines,
                                       G.ma_lhist_ready ? 1 : 0, ma_build_small());
  uint32_t c[4];
  HIPCHK(hipMemcpyAsync(c, G.d_lvl_ctr, sizeof c, hipMemcpyDeviceToHost, G.stream));
  k_lvl_decay<<<nb, B, 0, G.stream>>>(G.d_ma_lhist, npairs);
  HIPCHK(hipStreamSynchronize(G.stream));
  G.ma_level_lines = c[0];
  G.ma_level_small = std::min<int64_t>(c[1], G.build_list_cap);
  G.ma_level_large = std::min<int64_t>(c[3], G.build_list_cap - G.ma_level_small);
  G.ma_level_records = G.ma_level_small + G.ma_level_large;
  G.ma_initial_placement = !G.ma_lhist_ready;
  G.ma_lhist_ready = true;  // the transports from now on count
  return 0;
}

// the key records of the current level-mode placement (k_ma_build over the placement's list)
int ma_level_build(int nts) {
  const int64_t lds_small = std::min<int64_t>(G.ma_build_lds_doubles, ma_build_small());
  if (G.ma_level_small > 0)
    k_ma_build<<<(unsigned)std::min<int64_t>(G.ma_level_small, 1 << 16), 64, (size_t)std::max<int64_t>(1, lds_small) * 8,
                 G.stream>>>(G.K, G.d_build_list, (uint32_t)G.ma_level_small, nts);
  if (G.ma_level_large > 0)
    k_ma_build<<<(unsigned)std::min<int64_t>(G.ma_level_large, 1 << 16), 64,
                 (size_t)std::max<int64_t>(1, G.ma_build_lds_doubles) * 8, G.stream>>>(
        G.K, G.d_build_list + (G.build_list_cap - G.ma_level_large), (uint32_t)G.ma_level_large, nts);
  HIPCHK(hipGetLastError());
  return 0;
}

int64_t sum_i32(const int32_t *a, int n) {
  int64_t s = 0;
  for (int i = 0; i < n; i++) s += a[i];
  return s;
}

int check_kernel_error(const char *what) {
  int32_t err[4] = {0, 0, 0, 0};
  HIPCHK(hipMemcpy(err, G.K.E.err, sizeof(err), hipMemcpyDeviceToHost));
  if (err[0] != 0) {
    char buf[256];
    snprintf(buf, sizeof buf, "%s: device error code %d packet %d aux %d", what, err[0], err[1], err[2]);
    G.last_error = buf;
    return (err[0] == ERR_UNSUPPORTED_TYPE) ? ARTIS_ERR_UNSUPPORTED : ARTIS_ERR_PACKET_FAULT;
  }
  return 0;
}

// Device allocation with an optional injected failure (ARTIS_GPU_FAIL_ALLOC_ABOVE=<bytes>: any single request
// above that size fails as out-of-memory) so the error paths can be tested.
hipError_t dmalloc(void **p, size_t bytes) {
  *p = nullptr;
  if (const char *lim = getenv("ARTIS_GPU_FAIL_ALLOC_ABOVE"))
    if (bytes > (size_t)strtoull(lim, nullptr, 10)) return hipErrorOutOfMemory;
  return hipMalloc(p, bytes);
}

template <typename T>
void dfree(T *&p) {
  if (p) (void)hipFree((void *)p);
  p = nullptr;
}

// packet store + per-packet side state; after this every pointer is null and the capacity zero
void free_packets() {
  dfree(G.d_soa);
  dfree(G.d_aos);
  dfree(G.d_snapshot);
  G.have_snapshot = false;
  dfree(G.W.rng_n);
  dfree(G.W.pend);
  dfree(G.W.pend_jumps);
  dfree(G.W.ma_key);
  dfree(G.W.ma_sorted);
  dfree(G.W.ma_tick);
  dfree(G.W.ma_pre);
  dfree(G.W.mf_rec);
  for (int q = 0; q < NQUEUES; q++) dfree(G.W.q[q]);
  G.cap_pkts = 0;
  G.npkts = 0;
}

int alloc_packets(int64_t n) {
  if (n <= G.cap_pkts) return 0;
  free_packets();
  const size_t un = (size_t)n;
  struct Req {
    void **p;
    size_t bytes;
  };
  std::vector<Req> reqs = {{(void **)&G.d_soa, un * PKT_STORE_WORDS * 8},
                           {(void **)&G.d_aos, un * PKT_WORDS * 8},
                           {(void **)&G.W.rng_n, un * sizeof(uint32_t)},
                           {(void **)&G.W.pend, un * sizeof(int4)},
                           {(void **)&G.W.pend_jumps, un * sizeof(uint32_t)},
                           {(void **)&G.W.ma_key, un * sizeof(int32_t)},
                           {(void **)&G.W.ma_sorted, un * sizeof(int32_t)},
                           {(void **)&G.W.ma_tick, un * 2 * sizeof(int4)},
                           {(void **)&G.W.ma_pre, un * 2 * sizeof(int4)},
                           {(void **)&G.W.mf_rec, un * 2 * sizeof(int4)}};
  for (int q = 0; q < NQUEUES; q++) reqs.push_back({(void **)&G.W.q[q], un * sizeof(int32_t)});
  const int nreq = (int)reqs.size();
  for (int r = 0; r < nreq; r++) {
    const hipError_t e = dmalloc(reqs[r].p, reqs[r].bytes);
    if (e != hipSuccess) {
      G.last_error = std::string("packet store allocation (") + std::to_string(n) + " packets): " + hipGetErrorString(e);
      free_packets();
      return ARTIS_ERR_HIP;
    }
  }
  G.cap_pkts = n;
  return 0;
}

// Event-queue transport (wavefront.h): classify, then rounds of R -> M -> K kernels until both the R and M
// queues stay empty.  The host learns the queue sizes one round late (pinned async copies), so it never
// stalls the stream; a round enqueued after the work ran out finds empty queues and costs only its launches.
// the transport kernels read the context through a pointer to this device copy (physics.h)
int sync_ctx() {
  HIPCHK(hipStreamSynchronize(G.stream));
  HIPCHK(hipMemcpy(G.d_ctx, &G.K, sizeof(Ctx), hipMemcpyHostToDevice));
  return 0;
}

int tmark(int cls) {
  if (G.tev_used + 1 > G.tev.size()) {
    hipEvent_t e;
    HIPCHK(hipEventCreate(&e));
    G.tev.push_back(e);
    G.tev_class.push_back(cls);
  }
  G.tev_class[G.tev_used] = cls;
  HIPCHK(hipEventRecord(G.tev[G.tev_used++], G.stream));
  return 0;
}
// events come in (start, end) pairs; sum per class once the stream has drained
int tcollect() {
  for (int c = 0; c < ARTIS_KCLASS_COUNT; c++) {
    G.last_kernel_ms[c] = 0.;
    G.last_kernel_launches[c] = 0;
  }
  for (size_t i = 0; i + 1 < G.tev_used; i += 2) {
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, G.tev[i], G.tev[i + 1]));
    G.last_kernel_ms[G.tev_class[i]] += ms;
    G.last_kernel_launches[G.tev_class[i]]++;
  }
  G.tev_used = 0;
  return 0;
}
#define TSTART(c) \
  if (int rc_ = tmark(c)) return rc_
#define TEND(c) \
  if (int rc_ = tmark(c)) return rc_

// sort keys of the spawn records: propagation cell (high bits), then log nu_cmf in 4096 bins over [1e13, 1e17] Hz
__global__ void k_vpkt_keys(const double *__restrict__ spawn, uint32_t cap, uint32_t n, uint32_t *__restrict__ key,
                            uint32_t *__restrict__ idx) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n) return;
  const uint32_t where = (uint32_t)lo32(reinterpret_cast<const uint64_t *>(spawn)[11 * (uint64_t)cap + s]);
  const double nu = spawn[6 * (uint64_t)cap + s];
  const double f = log10(fmax(nu, 1e13) * 1e-13) * 0.25;  // [1e13, 1e17] -> [0, 1]
  const uint32_t b = (uint32_t)fmin(4095., fmax(0., f * 4095.));
  key[s] = (min(where, 0xfffffu) << 12) | b;  // (grids past 2^20 cells share the last cell key)
  idx[s] = s;
}

// virtual packets: trace the spawn records appended since the last flush, then empty the buffer
// (stream-ordered; the spawn count is read by the kernel itself)
int vpkt_flush() {
  if (!G.K.V.on) return 0;
  uint32_t ns = 0;
  const bool sort = G.vpkt_sort && G.d_vperm;
  if (sort) {
    // the trace order (DevVpkt::perm): a host round trip for the count, then a radix sort of (cell, nu) keys
    HIPCHK(hipMemcpyAsync(G.h_vcount, G.K.V.spawn_ctr, sizeof(uint32_t), hipMemcpyDeviceToHost, G.stream));
    HIPCHK(hipStreamSynchronize(G.stream));
    ns = std::min(*G.h_vcount, G.K.V.cap);
    if (ns == 0) {
      HIPCHK(hipMemsetAsync(G.K.V.spawn_ctr, 0, 2 * sizeof(uint32_t), G.stream));
      return 0;
    }
  }
  if (G.vev_used + 2 > G.vev.size()) {
    for (int k = 0; k < 2; k++) {
      hipEvent_t e;
      HIPCHK(hipEventCreate(&e));
      G.vev.push_back(e);
    }
  }
  HIPCHK(hipEventRecord(G.vev[G.vev_used++], G.stream));  // (the sort counts as virtual-packet time)
  if (sort) {
    k_vpkt_keys<<<(ns + 255) / 256, 256, 0, G.stream>>>(G.K.V.spawn, G.K.V.cap, ns, G.d_vkey, G.d_vidx);
    size_t tb = G.vsort_tmp_bytes;
    HIPCHK(hipcub::DeviceRadixSort::SortPairs(G.d_vsort_tmp, tb, G.d_vkey, G.d_vkey2, G.d_vidx, G.d_vperm, (int)ns,
                                              0, 32, G.stream));
  }
  // minimum waves per SIMD the virtual-packet kernel is compiled for (ARTIS_VPKT_OCC = 1, 2 or 3; more waves
  // hide more of the FP64 and memory latency of the walk at the price of register spills)
  static const int occ = [] {
    const char *e = getenv("ARTIS_VPKT_OCC");
    const int v = e ? atoi(e) : VPKT_OCC_DEFAULT;
    return (v == 2 || v == 3) ? v : 1;
  }();
  // every non-empty cell with a coefficient row: the kernel without the gather walk (whose PF-line prefetch arrays
  // would otherwise set the register allocation of the whole kernel); ARTIS_VPKT_LCONLY=0 forces the general one
  static const bool lc_ok = [] {
    const char *e = getenv("ARTIS_VPKT_LCONLY");
    return !(e && e[0] == '0');
  }();
  const bool lc_only = lc_ok && G.K.C.linecoef && G.K.C.linecoef_rows >= G.K.C.n_nonempty;
  // (at most 4 spectra at the default occupancy: the instance whose loops run over 4 spectra, not 8)
  if (lc_only && occ == 2 && G.K.V.nspectra <= 4)
    k_vpkt<0, 2, 4><<<(unsigned)G.wave_grid, WAVE_BLOCK, 0, G.stream>>>(G.d_ctx, G.W.refill_min);
  else if (lc_only && occ == 3)
    k_vpkt<0, 3><<<(unsigned)G.wave_grid, WAVE_BLOCK, 0, G.stream>>>(G.d_ctx, G.W.refill_min);
  else if (lc_only && occ == 2)
    k_vpkt<0, 2><<<(unsigned)G.wave_grid, WAVE_BLOCK, 0, G.stream>>>(G.d_ctx, G.W.refill_min);
  else if (lc_only)
    k_vpkt<0, 1><<<(unsigned)G.wave_grid, WAVE_BLOCK, 0, G.stream>>>(G.d_ctx, G.W.refill_min);
  else if (occ == 3)
    k_vpkt<VPKT_PF, 3><<<(unsigned)G.wave_grid, WAVE_BLOCK, 0, G.stream>>>(G.d_ctx, G.W.refill_min);
  else if (occ == 2)
    k_vpkt<VPKT_PF, 2><<<(unsigned)G.wave_grid, WAVE_BLOCK, 0, G.stream>>>(G.d_ctx, G.W.refill_min);
  else
    k_vpkt<VPKT_PF, 1><<<(unsigned)G.wave_grid, WAVE_BLOCK, 0, G.stream>>>(G.d_ctx, G.W.refill_min);
  HIPCHK(hipEventRecord(G.vev[G.vev_used++], G.stream));
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemsetAsync(G.K.V.spawn_ctr, 0, 2 * sizeof(uint32_t), G.stream));
  return 0;
}
// size the spawn buffer for n packets (artis_vpkt_params.spawn_capacity, default 16 per packet, >= 2^20)
int vpkt_prepare(int64_t n) {
  if (!G.K.V.on) return 0;
  // default: 16 spawns per packet, at most a quarter of the free HBM (a full buffer is traced and the launch
  // resumed, vpkt_drain), at least 2^20 records and never below the overflow records' count
  int64_t cap = G.vpkt_cap_param > 0 ? G.vpkt_cap_param : std::max<int64_t>(16 * n, 1 << 20);
  if (G.use_megakernel && G.vpkt_cap_param <= 0) {
    // the megakernel never parks a packet on a full buffer (only the split kernels resume, vpkt_drain): keep the
    // full 16 spawns per packet, or refuse the launch before it starts instead of overflowing inside it
    size_t freeb = 0, totalb = 0;
    (void)hipMemGetInfo(&freeb, &totalb);
    const double rec = VPKT_SPAWN_WORDS * sizeof(double) + 4 * sizeof(uint32_t);
    const double have = (double)G.vpkt_spawn_cap * rec;
    if ((double)cap * rec > 0.9 * ((double)freeb + have)) {
      G.last_error = "megakernel with virtual packets: " + std::to_string(cap) +
                     " spawn records (16 per packet) do not fit in free device memory; use the default (split-kernel) "
                     "engine or set the vpkt spawn_capacity";
      return ARTIS_ERR_UNSUPPORTED;
    }
  } else if (G.vpkt_cap_param <= 0) {
    size_t freeb = 0, totalb = 0;
    (void)hipMemGetInfo(&freeb, &totalb);
    const int64_t have = G.vpkt_spawn_cap;  // a buffer already held counts as free
    const double rec = VPKT_SPAWN_WORDS * sizeof(double) + 4 * sizeof(uint32_t);  // + the sort arrays
    const int64_t fit = (int64_t)((0.25 * (double)freeb) / rec) + have / 4;
    cap = std::max<int64_t>(std::min(cap, fit), 1 << 20);
  }
  cap = std::max<int64_t>(cap, G.K.V.ovf_cap);
  cap = std::min<int64_t>(cap, 0x7fffffff / 2);
  // k_vpkt's 32-bit fetch head runs over cap * nobs work items and overshoots by at most one wave per resident
  // wave: keep that below 2^32 so the head cannot wrap onto items already traced
  const int64_t overshoot = (int64_t)G.wave_grid * WAVE_BLOCK;
  cap = std::min<int64_t>(cap, (((int64_t)1 << 32) - 1 - overshoot) / std::max(1, G.K.V.nobs));
  if ((uint32_t)cap > G.vpkt_spawn_cap) {
    dfree(G.d_vpkt_spawn);
    G.vpkt_spawn_cap = 0;
    G.K.V.spawn = nullptr;
    G.K.V.cap = 0;
    HIPCHK(dmalloc((void **)&G.d_vpkt_spawn, (size_t)cap * VPKT_SPAWN_WORDS * sizeof(double)));
    G.vpkt_spawn_cap = (uint32_t)cap;
    const char *so = getenv("ARTIS_VPKT_SORT");
    G.vpkt_sort = !(so && so[0] == '0');
    for (uint32_t **a : {&G.d_vkey, &G.d_vkey2, &G.d_vidx, &G.d_vperm}) {
      dfree(*a);
      *a = nullptr;
    }
    dfree(G.d_vsort_tmp);
    G.d_vsort_tmp = nullptr;
    if (G.vpkt_sort) {
      for (uint32_t **a : {&G.d_vkey, &G.d_vkey2, &G.d_vidx, &G.d_vperm})
        HIPCHK(dmalloc((void **)a, (size_t)cap * sizeof(uint32_t)));
      G.vsort_tmp_bytes = 0;
      HIPCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, G.vsort_tmp_bytes, G.d_vkey, G.d_vkey2, G.d_vidx,
                                                G.d_vperm, (int)cap, 0, 32, G.stream));
      HIPCHK(dmalloc(&G.d_vsort_tmp, std::max<size_t>(G.vsort_tmp_bytes, 16)));
    }
  }
  if (!G.h_vcount) HIPCHK(hipHostMalloc((void **)&G.h_vcount, sizeof(uint32_t), hipHostMallocDefault));
  G.K.V.perm = G.vpkt_sort ? G.d_vperm : nullptr;
  G.K.V.spawn = G.d_vpkt_spawn;
  G.K.V.cap = G.vpkt_spawn_cap;
  HIPCHK(hipMemsetAsync(G.K.V.spawn_ctr, 0, 2 * sizeof(uint32_t), G.stream));
  HIPCHK(hipMemsetAsync(G.K.V.ovf_ctr, 0, sizeof(uint32_t), G.stream));
  HIPCHK(hipMemsetAsync(G.K.V.full, 0, sizeof(uint32_t), G.stream));
  G.vev_used = 0;
  G.vpkt_drains = 0;
  return 0;
}

// overflow records -> the front of the (just traced and emptied) spawn buffer; then the counters
__global__ void k_vpkt_ovf_copy(const double *__restrict__ ovf, uint32_t ovf_cap, const uint32_t *__restrict__ ovf_ctr,
                                double *__restrict__ spawn, uint32_t cap) {
  const uint64_t nrec = min(min(*ovf_ctr, ovf_cap), cap);
  const uint64_t total = nrec * VPKT_SPAWN_WORDS;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t w = i / nrec, s = i % nrec;
    spawn[w * cap + s] = ovf[w * ovf_cap + s];
  }
}
__global__ void k_vpkt_ovf_reset(uint32_t *ovf_ctr, uint32_t ovf_cap, uint32_t *spawn_ctr, uint32_t cap, uint32_t *full,
                                 uint32_t *qctr, const uint32_t *qsnap) {
  if (threadIdx.x == 0) {
    spawn_ctr[0] = min(min(*ovf_ctr, ovf_cap), cap);
    spawn_ctr[1] = 0;
    *ovf_ctr = 0;
    *full = 0;
    // the queue's untaken slots and the packets parked after its launch count: [min(head, count at launch), count)
    if (qctr) qctr[1] = min(qctr[1], *qsnap);
  }
}

// After a k_rpkt / k_kpkt launch over queue q: while its spawns filled the buffer, trace the buffer, move the
// overflow records to its front and resume the launch on the slots it left.  A host round trip per launch, paid
// only with virtual packets.
template <typename F>
int vpkt_drain(int q, F &&relaunch) {
  if (!G.K.V.on) return 0;
  while (true) {
    HIPCHK(hipMemcpyAsync(G.h_vfull, G.K.V.full, sizeof(uint32_t), hipMemcpyDeviceToHost, G.stream));
    HIPCHK(hipStreamSynchronize(G.stream));
    if (!*G.h_vfull) return 0;
    G.vpkt_drains++;
    if (int rc = vpkt_flush()) return rc;
    const DevVpkt &V = G.K.V;
    k_vpkt_ovf_copy<<<1024, 256, 0, G.stream>>>(V.ovf, V.ovf_cap, V.ovf_ctr, V.spawn, V.cap);
    k_vpkt_ovf_reset<<<1, 64, 0, G.stream>>>(V.ovf_ctr, V.ovf_cap, V.spawn_ctr, V.cap, V.full, G.W.ctr + 2 * q,
                                             G.d_qsnap);
    HIPCHK(hipMemcpyAsync(G.d_qsnap, G.W.ctr + 2 * q, sizeof(uint32_t), hipMemcpyDeviceToDevice, G.stream));
    HIPCHK(hipGetLastError());
    if (int rc = relaunch()) return rc;
  }
}
int vpkt_collect(const unsigned long long before[8]) {
  G.last_vpkt_ms = 0.;
  for (size_t i = 0; i + 1 < G.vev_used; i += 2) {
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, G.vev[i], G.vev[i + 1]));
    G.last_vpkt_ms += ms;
  }
  G.vev_used = 0;
  unsigned long long after[8];
  HIPCHK(hipMemcpy(after, G.K.V.ctr, sizeof(after), hipMemcpyDeviceToHost));
  G.last_vpkt_traces = (int64_t)(after[0] - before[0]);
  G.last_vpkt_spawns = (int64_t)(after[4] - before[4]);
  G.last_vpkt_work[0] = (int64_t)(after[5] - before[5]);
  G.last_vpkt_work[1] = (int64_t)(after[6] - before[6]);
  G.last_vpkt_work[2] = (int64_t)(after[7] - before[7]);
  G.last_vpkt_work[3] = (int64_t)((after[1] + after[2] + after[3]) - (before[1] + before[2] + before[3]));
#ifdef ARTIS_DIAG_VPKT_PASSES
  if (getenv("ARTIS_GPU_STATS")) {
    unsigned long long dg[16];
    HIPCHK(hipMemcpyFromSymbol(dg, HIP_SYMBOL(g_vpkt_diag), sizeof(dg)));
    fprintf(stderr, "[artis_gpu] k_vpkt (cumulative): wave passes %llu, busy lanes/pass %.1f, tracing lanes/pass %.1f, "
            "passes/refill %.1f, cycles/pass %.0f, refill cycles/pass %.0f\n", dg[0], (double)dg[1] / dg[0],
            (double)dg[2] / dg[0], (double)dg[0] / dg[3], (double)dg[4] / dg[0], (double)dg[5] / dg[0]);
    fprintf(stderr, "[artis_gpu] k_vpkt cycles/pass by phase: trace start %.0f, boundary + continuum %.0f, line walk %.0f, "
            "segment end %.0f, escape %.0f\n", (double)dg[6] / dg[0], (double)dg[7] / dg[0], (double)dg[8] / dg[0],
            (double)dg[9] / dg[0], (double)dg[10] / dg[0]);
  }
#endif
  return 0;
}

#define WAVE_MAX_ROUNDS 10000000
int run_wavefront(int64_t n, int nts, double t2) {
  WaveState W = G.W;
  if (!(G.K.C.have_macache && W.ma_binned)) W.ma_tick = nullptr;  // tickets: cached walk over the binned queue
  if (!W.ma_tick || !G.ma_pre_on) W.ma_pre = nullptr;            // pre-tickets written by the queue's producers
  if (!G.mf_rec_on) W.mf_rec = nullptr;                           // F-queue records (else pend / pend_jumps / rng_n)
  // the M queue's producers bin it as they append (many cells only: the block-local binning of few-cell models
  // counts in LDS; not with the binned R queue, which uses the same counts array)
  W.bin_push = W.ma_binned && G.bin_push_on && !G.r_binned && G.K.C.n_nonempty > 0 &&
               !(G.ma_bin_blk && G.K.C.n_nonempty + 1 <= MA_BIN_LDS);
  const unsigned grid = (unsigned)G.wave_grid;
  if (int rc = sync_ctx()) return rc;
  G.tev_used = 0;
  HIPCHK(hipMemsetAsync(W.stats, 0, 48 * sizeof(unsigned long long), G.stream));
  HIPCHK(hipMemsetAsync(W.ctr, 0, NQUEUES * 2 * sizeof(uint32_t), G.stream));
  if (W.bin_push) HIPCHK(hipMemsetAsync(W.bins, 0, (size_t)(G.K.C.n_nonempty + 1) * sizeof(uint32_t), G.stream));
  TSTART(3);
  k_classify<<<(unsigned)((n + WAVE_BLOCK - 1) / WAVE_BLOCK), WAVE_BLOCK, 0, G.stream>>>(G.d_ctx, W, G.d_soa, n, t2);
  if (G.K.T.g_nlines) {  // pellets / gammas / leptons -> k-packets ahead of the rounds (counted with classify)
    k_gamma<<<grid / 4, WAVE_BLOCK, 0, G.stream>>>(G.d_ctx, W, G.d_soa, n, nts, t2);
  }
  TEND(3);
  HIPCHK(hipGetLastError());
  int64_t round = 0;
  bool done = false;
  // the QX queue's length at the end of the round before last, as the host last read it (-1: not read yet)
  int64_t qx_known = -1;
  const bool first_placement = G.ma_initial_placement;
  for (; round < WAVE_MAX_ROUNDS && !done; round++) {
    // level mode: after the first rounds of a transport on the initial placement (and again a few rounds later),
    // the records go to the pairs the walks have used so far (the rest of the timestep's walks use them;
    // placement never changes a result).
    // Between rounds no ticket holds a record line: k_ma_scatter looks them up again below.
    if (G.K.C.ma_level_mode && first_placement && (round == 2 || round == 8)) {
      if (int rc = ma_level_place()) return rc;
      if (int rc = ma_level_build(nts)) return rc;
    }
    // waves per SIMD k_rpkt is compiled for (ARTIS_GPU_RPKT_OCC = 1, 2 or 3).  The r-packet step needs ~300
    // registers; at 1 wave/SIMD nothing hides its FP64 latency, and forcing 2 (spilling to scratch) measured
    // 1.80 s -> 1.53 s per bench step on MI355X, so 2 is the default.
    static const int rpkt_occ = [] {
      const char *e = getenv("ARTIS_GPU_RPKT_OCC");
      return (e && (e[0] == '1' || e[0] == '3')) ? e[0] - '0' : 2;
    }();
    // the R queue binned by cell (ARTIS_GPU_R_BIN=1; default queue order); not with virtual packets, whose resumed
    // launches read parked packets appended to the queue itself
    W.r_binned = G.r_binned && !G.K.V.on && G.K.C.n_nonempty > 0;
    if (W.r_binned) {
      TSTART(4);
      const int nne = G.K.C.n_nonempty;
      HIPCHK(hipMemsetAsync(W.bins, 0, (size_t)(nne + 1) * sizeof(uint32_t), G.stream));
      k_r_bin<<<grid, WAVE_BLOCK, 0, G.stream>>>(G.d_ctx, W, G.d_soa);
      HIPCHK(hipcub::DeviceScan::ExclusiveSum(G.d_scan_tmp, G.scan_tmp_bytes, W.bins, G.d_binoffs, nne + 1,
                                              G.stream));
      k_r_scatter<<<grid, WAVE_BLOCK, 0, G.stream>>>(G.d_ctx, W, G.d_binoffs);
      TEND(4);
    }
    // the per-block estimator accumulator of few-cell models (dynamic LDS, sized only when it is used)
    const size_t est_shm = est_lds_on(G.K) ? EST_LDS_DOUBLES * sizeof(double) : 0;
    // detailed bf estimators (the nebular options): the instance whose continuum sums are made by the whole wave
    const bool rpkt_coop = G.K.R.detailed_bf && G.K.T.nbf > 0 && G.K.R.do_r_lc && G.rpkt_coop;
    // the bounded line walk (k_rpkt WALK) when the previous transport's steps scanned more than 8 lines each on
    // average (ARTIS_GPU_RPKT_WALK=1 / 0 forces it on / off)
    const bool rpkt_walk =
        G.rpkt_walk > 0 ||
        (G.rpkt_walk < 0 && G.last_work[WK_RPKT_STEPS] > 0 && G.last_work[WK_LINES_SCANNED] > 8 * G.last_work[WK_RPKT_STEPS]);
    auto launch_rpkt = [&]() -> int {
      if (rpkt_coop)
        k_rpkt<2, true><<<grid, WAVE_BLOCK, est_shm, G.stream>>>(G.d_ctx, W, G.d_soa, n, nts, t2);
      else if (rpkt_walk)
        k_rpkt<2, false, RPKT_WALK_LINES><<<grid, WAVE_BLOCK, est_shm, G.stream>>>(G.d_ctx, W, G.d_soa, n, nts, t2);
      else if (rpkt_occ == 3)
        k_rpkt<3, false><<<grid, WAVE_BLOCK, est_shm, G.stream>>>(G.d_ctx, W, G.d_soa, n, nts, t2);
      else if (rpkt_occ == 2)
        k_rpkt<2, false><<<grid, WAVE_BLOCK, est_shm, G.stream>>>(G.d_ctx, W, G.d_soa, n, nts, t2);
      else
        k_rpkt<1, false><<<grid, WAVE_BLOCK, est_shm, G.stream>>>(G.d_ctx, W, G.d_soa, n, nts, t2);
      return 0;
    };
    if (G.K.V.on)
      HIPCHK(hipMemcpyAsync(G.d_qsnap, W.ctr + 2 * QR, sizeof(uint32_t), hipMemcpyDeviceToDevice, G.stream));
    TSTART(0);
    if (int rc = launch_rpkt()) return rc;
    TEND(0);
    W.r_binned = 0;
    if (int rc = vpkt_drain(QR, [&]() -> int {
          TSTART(0);
          if (int rc2 = launch_rpkt()) return rc2;
          TEND(0);
          return 0;
        }))
      return rc;
    HIPCHK(hipMemsetAsync(W.ctr + 2 * QR, 0, 2 * sizeof(uint32_t), G.stream));
    TSTART(4);  // class 4: the macro-atom queue binning (class 1 is k_ma alone)
    if (W.ma_binned) {
      const int nne = G.K.C.n_nonempty;
      // few cells: block-local counts (one device atomic per block and bin instead of one per queue entry)
      const bool blk = G.ma_bin_blk && nne + 1 <= MA_BIN_LDS;
      if (!W.bin_push) {
        HIPCHK(hipMemsetAsync(W.bins, 0, (size_t)(nne + 1) * sizeof(uint32_t), G.stream));
        if (blk)
          k_ma_bin_blk<<<grid, WAVE_BLOCK, 0, G.stream>>>(G.d_ctx, W, G.d_soa);
        else
          k_ma_bin<<<grid, WAVE_BLOCK, 0, G.stream>>>(G.d_ctx, W, G.d_soa);
      }
      HIPCHK(hipcub::DeviceScan::ExclusiveSum(G.d_scan_tmp, G.scan_tmp_bytes, W.bins, G.d_binoffs, nne + 1,
                                              G.stream));
      // (the counts are the scan's input only: the next round's appends -- k_ma_exact's and k_kpkt's in this
      // round, then k_rpkt's -- count from zero)
      if (W.bin_push) HIPCHK(hipMemsetAsync(W.bins, 0, (size_t)(nne + 1) * sizeof(uint32_t), G.stream));
      if (blk)
        k_ma_scatter_blk<<<grid, WAVE_BLOCK, 0, G.stream>>>(G.d_ctx, W, G.d_soa, n, G.d_binoffs);
      else
        k_ma_scatter<<<grid, WAVE_BLOCK, 0, G.stream>>>(G.d_ctx, W, G.d_soa, n, G.d_binoffs);
    }
    HIPCHK(hipMemsetAsync(W.xhead, 0, 8 * sizeof(uint32_t), G.stream));
    TEND(4);
    TSTART(1);
    // ARTIS_GPU_MA_WAVES=w (default 4): launch only w blocks per CU (w resident waves per SIMD) -- fewer
    // concurrent walks thrash the caches less; the walk is bound by the memory system, not by latency hiding
    // (1e7-packet bench: 2 waves 4694 ms, 3: 3761 ms, 4: 3317 ms, 8: 3725 ms; profiles/r02_ab_ma_waves.txt)
    static const int ma_waves = [] {
      const char *e = getenv("ARTIS_GPU_MA_WAVES");
      const int v = e ? atoi(e) : 4;
      return (v >= 1 && v <= 8) ? v : 4;
    }();
    const unsigned ma_grid = ma_waves ? (unsigned)(G.wave_grid / 8 * ma_waves) : grid;
    if (G.K.C.ma_level_mode)
      // (the whole-cell placement before the first transport covers few of the pairs walked: those walks would
      // take a round per parked jump, so the first transport makes its exact-sum jumps inline)
      if (G.ma_level_coop || first_placement)
        k_ma<4, true, true><<<ma_grid, WAVE_BLOCK, 0, G.stream>>>(G.d_ctx, W, G.d_soa, n, nts);
      else
        k_ma<8, false, true><<<ma_grid, WAVE_BLOCK, 0, G.stream>>>(G.d_ctx, W, G.d_soa, n, nts);
    else if (G.ma_occ == 8)
      k_ma<8, false, false><<<ma_grid, WAVE_BLOCK, 0, G.stream>>>(G.d_ctx, W, G.d_soa, n, nts);
    else
      k_ma<1, false, false><<<ma_grid, WAVE_BLOCK, 0, G.stream>>>(G.d_ctx, W, G.d_soa, n, nts);
    TEND(1);
    HIPCHK(hipMemsetAsync(W.ctr + 2 * QM, 0, 2 * sizeof(uint32_t), G.stream));
    // jumps the 32-bit keys could not decide (rare), exact; walks go back to M.  Launched only when the queue may
    // hold any: in the first two rounds, and whenever the host's last reading (the round before last) found entries.
    // A round without the launch leaves its entries queued (QX is reset only after a launch) for a later one; the
    // loop does not end while QX holds any.
    if (round < 2 || qx_known != 0) {
      TSTART(5);
      // (one wave per block and queue entry, 2 waves per SIMD: the 256-VGPR kernel's limit.  A quarter of that grid
      // left half the SIMDs without a wave, and the exact jumps of a large atom's level mode are latency chains)
      k_ma_exact<<<grid, 64, 0, G.stream>>>(G.d_ctx, W, G.d_soa, n, nts);
      TEND(5);
      HIPCHK(hipMemsetAsync(W.ctr + 2 * QX, 0, 2 * sizeof(uint32_t), G.stream));
    }
    {  // the walks' deactivations -> R / K
      TSTART(6);
      if (G.K.V.on)
        HIPCHK(hipMemcpyAsync(G.d_qsnap, W.ctr + 2 * QF, sizeof(uint32_t), hipMemcpyDeviceToDevice, G.stream));
      k_ma_finish<<<grid / 4, WAVE_BLOCK, 0, G.stream>>>(G.d_ctx, W, G.d_soa, n, nts, t2);
      TEND(6);
      if (int rc = vpkt_drain(QF, [&]() -> int {
            TSTART(6);
            k_ma_finish<<<grid / 4, WAVE_BLOCK, 0, G.stream>>>(G.d_ctx, W, G.d_soa, n, nts, t2);
            TEND(6);
            return 0;
          }))
        return rc;
      HIPCHK(hipMemsetAsync(W.ctr + 2 * QF, 0, 2 * sizeof(uint32_t), G.stream));
    }
    if (G.K.V.on)
      HIPCHK(hipMemcpyAsync(G.d_qsnap, W.ctr + 2 * QK, sizeof(uint32_t), hipMemcpyDeviceToDevice, G.stream));
    TSTART(2);
    k_kpkt<<<grid / 4, WAVE_BLOCK, 0, G.stream>>>(G.d_ctx, W, G.d_soa, n, nts, t2);
    TEND(2);
    if (int rc = vpkt_drain(QK, [&]() -> int {
          TSTART(2);
          k_kpkt<<<grid / 4, WAVE_BLOCK, 0, G.stream>>>(G.d_ctx, W, G.d_soa, n, nts, t2);
          TEND(2);
          return 0;
        }))
      return rc;
    HIPCHK(hipMemsetAsync(W.ctr + 2 * QK, 0, 2 * sizeof(uint32_t), G.stream));
    if (int rc = vpkt_flush()) return rc;
    HIPCHK(hipGetLastError());
    const int slot = (int)(round & 1);
    HIPCHK(hipMemcpyAsync(G.h_ctr + slot * NQUEUES * 2, W.ctr, NQUEUES * 2 * sizeof(uint32_t),
                          hipMemcpyDeviceToHost, G.stream));
    HIPCHK(hipEventRecord(G.ev_round[slot], G.stream));
    if (round > 0) {
      const int prev = (int)((round - 1) & 1);
      HIPCHK(hipEventSynchronize(G.ev_round[prev]));
      const uint32_t *c = G.h_ctr + prev * NQUEUES * 2;
      qx_known = c[2 * QX];
      if (c[2 * QR] == 0 && c[2 * QM] == 0 && c[2 * QX] == 0) done = true;
    }
  }
  if (!done) {
    // the loop hit its cap: check the last round before declaring a stall
    HIPCHK(hipStreamSynchronize(G.stream));
    const uint32_t *c = G.h_ctr + ((round - 1) & 1) * NQUEUES * 2;
    if (c[2 * QR] != 0 || c[2 * QM] != 0 || c[2 * QX] != 0) {
      G.last_error = "wavefront transport did not converge";
      return ARTIS_ERR_PACKET_FAULT;
    }
  }
  G.last_rounds = round;
  HIPCHK(hipStreamSynchronize(G.stream));
  if (getenv("ARTIS_GPU_STATS")) {
    unsigned long long st[48];
    HIPCHK(hipMemcpy(st, W.stats, sizeof(st), hipMemcpyDeviceToHost));
    const char *nm[2] = {"rpkt", "ma"};
    for (int c = 0; c < 2; c++)
      fprintf(stderr,
              "[artis_gpu] %s: wave passes %llu, lane utilisation %.3f, cycles/pass %.0f, passes/refill %.1f, "
              "cycles/refill %.0f, step cycles/pass %.0f\n",
              nm[c], st[4 * c], st[4 * c] ? (double)st[4 * c + 1] / (64.0 * st[4 * c]) : 0.,
              st[4 * c] ? (double)st[4 * c + 2] / st[4 * c] : 0., st[4 * c + 3] ? (double)st[4 * c] / st[4 * c + 3] : 0.,
              st[4 * c + 3] ? (double)st[16 + 4 * c] / st[4 * c + 3] : 0.,
              st[4 * c] ? (double)st[17 + 4 * c] / st[4 * c] : 0.);
    fprintf(stderr,
            "[artis_gpu] rpkt per pass: lines scanned wave-max %.2f vs lane-mean %.3f; bf continua wave-max %.2f vs "
            "lane-mean %.3f\n",
            st[0] ? (double)st[24] / st[0] : 0., st[0] ? (double)st[25] / (64.0 * st[0]) : 0.,
            st[0] ? (double)st[26] / st[0] : 0., st[0] ? (double)st[27] / (64.0 * st[0]) : 0.);
    fprintf(stderr, "[artis_gpu] macro-atom jumps made with the exact sums (undecided 32-bit keys): %llu\n", st[40]);
    if (st[32] + st[33] + st[34] + st[35] + st[36])
      fprintf(stderr,
              "[artis_gpu] rpkt step phases (cycles/pass): boundary %.0f, kappa %.0f, line loop %.0f, move+estimators "
              "%.0f, event %.0f, wave continuum sums %.0f\n",
              (double)st[32] / st[0], (double)st[33] / st[0], (double)st[34] / st[0], (double)st[35] / st[0],
              (double)st[36] / st[0], (double)st[37] / st[0]);
#ifdef ARTIS_STAMPS
    {
      unsigned long long dg[48];
      HIPCHK(hipMemcpyFromSymbol(dg, HIP_SYMBOL(g_ma_diag), sizeof(dg)));
      for (int a = 0; a < ARTIS_MA_ACTION_COUNT; a++)
        fprintf(stderr, "[artis_gpu] ma action %d: searches %llu, pending %llu, probes %llu\n", a, dg[a], dg[16 + a],
                dg[32 + a]);
      if (dg[9])
        fprintf(stderr,
                "[artis_gpu] ma up-same selections of blocked arrays %llu: in the line-0 suffix %llu, first 16 %llu, "
                "last 16 %llu, first suffix-size %llu, mean size %.1f, mean suffix %.1f, quarters %llu %llu %llu %llu\n",
                dg[9], dg[10], dg[11], dg[12], dg[13], (double)dg[14] / dg[9], (double)dg[15] / dg[9], dg[25], dg[26],
                dg[27], dg[28]);
      if (dg[43])
        fprintf(stderr, "[artis_gpu] ma step sections (cycles per wave step): action keys %.0f, search %.0f, rest %.0f\n",
                (double)dg[40] / dg[43], (double)dg[41] / dg[43], (double)dg[42] / dg[43]);
    }
#endif
    if (st[41] + st[42] + st[43])
      fprintf(stderr, "[artis_gpu] ma pass phases (cycles/pass): fetch %.0f, jump %.0f, rest %.0f, load wait %.0f\n",
              (double)st[41] / st[4], (double)st[42] / st[4], (double)st[43] / st[4], (double)st[44] / st[4]);
  }
  return tcollect();
}

}  // namespace

// ============================================================================================== C ABI
extern "C" {


}  // extern "C"

// ============================================================================ update_grid temperature solution
// artis_gpu_solve_temperatures (include/artis_gpu.h, te_solver.h): every caller array is copied in, the solution
// is computed for the listed cells and every array is copied back, so cells not listed round-trip unchanged.
namespace {
struct DevBufs {
  std::vector<void *> p;
  ~DevBufs() {
    for (void *q : p) (void)hipFree(q);
  }
  template <typename T>
  int get(T **d, size_t count, const T *src) {
    if (count == 0) count = 1;
    HIPCHK(hipMalloc((void **)d, count * sizeof(T)));
    p.push_back((void *)*d);
    // host-synchronous: a pageable source may be a temporary, and an asynchronous copy queued behind running
    // kernels would read it after it is gone
    if (src) HIPCHK(hipMemcpy(*d, src, count * sizeof(T), hipMemcpyHostToDevice));
    return 0;
  }
};
template <typename T>
int d2h_vec(std::vector<T> &h, const T *d, size_t n) {
  h.assign(n, T());
  if (n) HIPCHK(hipMemcpy(h.data(), d, n * sizeof(T), hipMemcpyDeviceToHost));
  return 0;
}
}  // namespace

extern "C" {
int artis_gpu_solve_temperatures(const artis_te_tables *tab, const artis_te_params *par, artis_te_cells *c) {
  if (!G.initialised) return ARTIS_ERR_NOT_INITIALISED;
  const DevRun &R = G.K.R;
  if (R.nlte_on || R.no_lut_photoion || R.no_lut_bfheating || R.nt_on) {
    G.last_error = "solve_temperatures: only the LTE-population options (NLTE_POPS_ON, NO_LUT_*, NT_ON false)";
    return ARTIS_ERR_UNSUPPORTED;
  }
  if (!tab || !par || !c || !tab->bfheating_coeff || !tab->ion_alpha_sp || c->ncells < 0 || (c->ncells > 0 && !c->mgi) ||
      !c->TR || !c->W || !c->TJ || !c->rho || !c->thick || !c->elem_abundance || !c->elem_meanweight || !c->vol_init ||
      !c->ffheatingestimator || !c->colheatingestimator || !c->gammaestimator || !c->bfheatingestimator || !c->Te ||
      !c->groundlevelpop || !c->nne || !c->nnetot || !c->partfunct || !c->totalcooling || !c->cooling_contrib_ion ||
      !(par->T_min > 0. && par->T_max > par->T_min && par->accuracy > 0. && par->tmin > 0. && par->t_current > 0.)) {
    G.last_error = "solve_temperatures: NULL table / cell array or bad parameters";
    return ARTIS_ERR_BAD_ARGUMENT;
  }
  const int np = G.npts_model, ne = G.nelements, ni = G.nions_total, nmx = G.maxnions;
  const DevTab &T = G.K.T;
  for (int k = 0; k < c->ncells; k++)
    if (c->mgi[k] < 0 || c->mgi[k] >= np) {
      G.last_error = "solve_temperatures: cell index out of range";
      return ARTIS_ERR_BAD_ARGUMENT;
    }
  if (c->ncells == 0) return 0;
  // the heating sum's level list (thermalbalance.cc:304-310): ionising levels of every ion but the top one
  std::vector<int32_t> nions, uoff, ionis, ul0;
  if (d2h_vec(nions, T.elem_nions, ne) || d2h_vec(uoff, T.elem_uniqueionoffset, ne) ||
      d2h_vec(ionis, T.ion_ionisinglevels, ni) || d2h_vec(ul0, T.ion_uniqueleveloffset, ni))
    return ARTIS_ERR_HIP;
  std::vector<int32_t> hb;
  for (int e = 0; e < ne; e++) {
    if (nions[e] > TE_MAX_IONS_PER_ELEMENT) {
      G.last_error = "solve_temperatures: more ions per element than TE_MAX_IONS_PER_ELEMENT";
      return ARTIS_ERR_UNSUPPORTED;
    }
    for (int i = 0; i < nions[e] - 1; i++)
      for (int l = 0; l < ionis[uoff[e] + i]; l++) hb.push_back(ul0[uoff[e] + i] + l);
  }
  DevBufs B;
  TeDev D{};
  const size_t npf = (size_t)np, npi = (size_t)np * ni, npe = (size_t)np * ne, npg = (size_t)np * ne * nmx;
  int rc = 0;
  rc |= B.get((double **)&D.bfheat_lut, (size_t)T.tablesize * T.nbf, tab->bfheating_coeff);
  rc |= B.get((float **)&D.alpha_sp, (size_t)ni * T.tablesize, tab->ion_alpha_sp);
  rc |= B.get((int32_t **)&D.anumber, (size_t)ne, G.h_anumber.data());
  rc |= B.get((int32_t **)&D.hb_ul, hb.size(), hb.data());
  rc |= B.get((int32_t **)&D.mgi, (size_t)c->ncells, c->mgi);
  rc |= B.get((float **)&D.TR, npf, c->TR);
  rc |= B.get((float **)&D.W, npf, c->W);
  rc |= B.get((float **)&D.TJ, npf, c->TJ);
  rc |= B.get((float **)&D.rho, npf, c->rho);
  rc |= B.get((int16_t **)&D.thick, npf, c->thick);
  rc |= B.get((float **)&D.abund, npe, c->elem_abundance);
  rc |= B.get((float **)&D.meanw, npe, c->elem_meanweight);
  rc |= B.get((double **)&D.vol, npf, c->vol_init);
  rc |= B.get((double **)&D.ffheat, npf, c->ffheatingestimator);
  rc |= B.get((double **)&D.colheat, npf, c->colheatingestimator);
  rc |= B.get((double **)&D.gamma, npg, c->gammaestimator);
  rc |= B.get((double **)&D.bfest, npg, c->bfheatingestimator);
  if (c->heating_dep) rc |= B.get((double **)&D.hdep, npf, c->heating_dep);
  rc |= B.get(&D.Te, npf, c->Te);
  rc |= B.get(&D.gp, npi, c->groundlevelpop);
  rc |= B.get(&D.nne, npf, c->nne);
  rc |= B.get(&D.nnetot, npf, c->nnetot);
  rc |= B.get(&D.pf, npi, c->partfunct);
  rc |= B.get(&D.totcool, npf, c->totalcooling);
  rc |= B.get(&D.ccion, npi, c->cooling_contrib_ion);
  if (c->heatingcoolingrates) rc |= B.get(&D.rates, npf * ARTIS_TE_NRATES, (const double *)c->heatingcoolingrates);
  if (c->te_iterations) rc |= B.get(&D.iters, npf, (const int32_t *)c->te_iterations);
  rc |= B.get(&D.upp, npe, (const int32_t *)nullptr);
  rc |= B.get(&D.hbc, hb.size() * (size_t)c->ncells, (const double *)nullptr);
  rc |= B.get(&D.fail, 1, (const int32_t *)nullptr);
  if (rc) return ARTIS_ERR_HIP;
  HIPCHK(hipMemsetAsync(D.fail, 0, sizeof(int32_t), G.stream));
  D.nhb = (int32_t)hb.size();
  D.ncells = c->ncells;
  D.t_current = par->t_current;
  D.tmin = par->tmin;
  D.T_min = par->T_min;
  D.T_max = par->T_max;
  D.accuracy = par->accuracy;
  D.initial_iteration = par->initial_iteration;
  D.direct_col_heat = par->direct_col_heat;
  HIPCHK(hipEventRecord(G.ev0, G.stream));
  if (D.nhb > 0) {
    const int64_t nw = (int64_t)D.nhb * D.ncells;
    k_te_bfheat<<<(unsigned)((nw + 255) / 256), 256, 0, G.stream>>>(G.K, D);
  }
  // lanes per cell: one per ion for the per-ion collisional-excitation sums of the cooling rate (te_cooling_rates),
  // floor(64 / g) cells per wave (12 ions: 5 cells on 60 lanes); ARTIS_GPU_TE_LANES overrides (1 = one cell per lane)
  int g = te_lanes_per_cell(ni);
  if (const char *ev = getenv("ARTIS_GPU_TE_LANES")) {
    const int v = atoi(ev);
    if (v >= 1 && v <= 64) g = v;
  }
  const int cpw = 64 / g;
  Ctx *dK = nullptr;
  TeDev *dD = nullptr;
  if (B.get(&dK, 1, &G.K) || B.get(&dD, 1, &D)) return ARTIS_ERR_HIP;
  k_te_solve<<<(unsigned)((D.ncells + cpw - 1) / cpw), 64, (size_t)cpw * ni * sizeof(double), G.stream>>>(dK, dD, g);
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(G.ev1, G.stream));
  HIPCHK(hipEventSynchronize(G.ev1));
  float ms = 0.f;
  HIPCHK(hipEventElapsedTime(&ms, G.ev0, G.ev1));
  G.last_te_ms = ms;
  int32_t fail = 0;
  HIPCHK(hipMemcpy(&fail, D.fail, sizeof(int32_t), hipMemcpyDeviceToHost));
  if (fail) {
    // the caller's cell state is left as it was: the reference aborts before writing a partial solution
    char buf[160];
    snprintf(buf, sizeof buf,
             "solve_temperatures: a GSL root-finder error (endpoints do not straddle zero / non-finite value) in "
             "model cell %d -- the reference aborts here",
             fail - 1);
    G.last_error = buf;
    return ARTIS_ERR_PACKET_FAULT;
  }
  HIPCHK(hipMemcpy(c->Te, D.Te, npf * sizeof(float), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(c->groundlevelpop, D.gp, npi * sizeof(float), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(c->nne, D.nne, npf * sizeof(float), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(c->nnetot, D.nnetot, npf * sizeof(float), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(c->partfunct, D.pf, npi * sizeof(float), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(c->totalcooling, D.totcool, npf * sizeof(double), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(c->cooling_contrib_ion, D.ccion, npi * sizeof(double), hipMemcpyDeviceToHost));
  if (c->heatingcoolingrates)
    HIPCHK(hipMemcpy(c->heatingcoolingrates, D.rates, npf * ARTIS_TE_NRATES * sizeof(double), hipMemcpyDeviceToHost));
  if (c->te_iterations) HIPCHK(hipMemcpy(c->te_iterations, D.iters, npf * sizeof(int32_t), hipMemcpyDeviceToHost));
  return 0;
}
double artis_gpu_last_te_ms(void) { return G.last_te_ms; }

int artis_gpu_prepare_temperatures(const artis_te_tables *tab, const artis_te_params *par, const artis_ug_prepare *pr,
                                   const artis_te_cells *c) {
  if (!G.initialised) return ARTIS_ERR_NOT_INITIALISED;
  const DevRun &R = G.K.R;
  if (R.nlte_on || R.no_lut_photoion || R.no_lut_bfheating || R.nt_on) {
    G.last_error = "prepare_temperatures: only the LTE-population options (NLTE_POPS_ON, NO_LUT_*, NT_ON false)";
    return ARTIS_ERR_UNSUPPORTED;
  }
  if (!tab || !par || !pr || !c || !tab->bfheating_coeff || c->ncells < 0 || (c->ncells > 0 && !c->mgi) || !c->TR ||
      !c->W || !c->TJ || !c->Te || !c->rho || !c->thick || !c->elem_abundance || !c->vol_init || !c->groundlevelpop ||
      !pr->J || !pr->nuJ || !pr->ffheating || !pr->colheating || !pr->gammaestimator || !pr->bfheatingestimator ||
      !pr->nne || !pr->TR_out || !pr->W_out || !pr->TJ_out || !pr->ffheating_out ||
      !pr->colheating_out || !pr->gamma_out || !pr->bfheating_out || !pr->corrphotoionrenorm_out ||
      !(pr->deltat > 0. && pr->tratmid > 0. && pr->nprocs > 0 && par->T_max > par->T_min && par->T_min > 0.)) {
    G.last_error = "prepare_temperatures: NULL array or bad parameters";
    return ARTIS_ERR_BAD_ARGUMENT;
  }
  const int np = G.npts_model, ne = G.nelements, ni = G.nions_total, nmx = G.maxnions;
  for (int k = 0; k < c->ncells; k++)
    if (c->mgi[k] < 0 || c->mgi[k] >= np) {
      G.last_error = "prepare_temperatures: cell index out of range";
      return ARTIS_ERR_BAD_ARGUMENT;
    }
  if (c->ncells == 0) return 0;
  const size_t npf = (size_t)np, npi = (size_t)np * ni, npe = (size_t)np * ne, npg = (size_t)np * ne * nmx;
  DevBufs B;
  UgDev U{};
  int rc = 0;
  rc |= B.get((int32_t **)&U.mgi, (size_t)c->ncells, c->mgi);
  rc |= B.get((float **)&U.TR, npf, c->TR);
  rc |= B.get((float **)&U.W, npf, c->W);
  rc |= B.get((float **)&U.TJ, npf, c->TJ);
  rc |= B.get((float **)&U.Te, npf, (const float *)c->Te);
  rc |= B.get((float **)&U.nne, npf, pr->nne);
  rc |= B.get((float **)&U.gp, npi, (const float *)c->groundlevelpop);
  rc |= B.get((float **)&U.rho, npf, c->rho);
  rc |= B.get((float **)&U.abund, npe, c->elem_abundance);
  rc |= B.get((int16_t **)&U.thick, npf, c->thick);
  rc |= B.get((double **)&U.vol, npf, c->vol_init);
  rc |= B.get((double **)&U.J, npf, pr->J);
  rc |= B.get((double **)&U.nuJ, npf, pr->nuJ);
  rc |= B.get((double **)&U.ff, npf, pr->ffheating);
  rc |= B.get((double **)&U.col, npf, pr->colheating);
  rc |= B.get((double **)&U.gam, npg, pr->gammaestimator);
  rc |= B.get((double **)&U.bfh, npg, pr->bfheatingestimator);
  rc |= B.get((double **)&U.bfheat_lut, (size_t)G.K.T.tablesize * G.K.T.nbf, tab->bfheating_coeff);
  rc |= B.get(&U.TR_out, npf, (const float *)pr->TR_out);
  rc |= B.get(&U.W_out, npf, (const float *)pr->W_out);
  rc |= B.get(&U.TJ_out, npf, (const float *)pr->TJ_out);
  rc |= B.get(&U.ff_out, npf, (const double *)pr->ffheating_out);
  rc |= B.get(&U.col_out, npf, (const double *)pr->colheating_out);
  rc |= B.get(&U.gam_out, npg, (const double *)pr->gamma_out);
  rc |= B.get(&U.bfh_out, npg, (const double *)pr->bfheating_out);
  rc |= B.get(&U.renorm_out, npg, (const double *)pr->corrphotoionrenorm_out);
  rc |= B.get(&U.fail, 1, (const int32_t *)nullptr);
  if (rc) return ARTIS_ERR_HIP;
  HIPCHK(hipMemsetAsync(U.fail, 0, sizeof(int32_t), G.stream));
  U.ncells = c->ncells;
  U.nprocs = pr->nprocs;
  U.initial_iteration = par->initial_iteration;
  U.deltat = pr->deltat;
  U.tratmid = pr->tratmid;
  U.T_min = par->T_min;
  U.T_max = par->T_max;
  Ctx *dK = nullptr;
  UgDev *dU = nullptr;
  if (B.get(&dK, 1, &G.K) || B.get(&dU, 1, &U)) return ARTIS_ERR_HIP;
  k_ug_prepare<<<(unsigned)((U.ncells + 255) / 256), 256, 0, G.stream>>>(dK, dU);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(G.stream));
  int32_t fail = 0;
  HIPCHK(hipMemcpy(&fail, U.fail, sizeof(int32_t), hipMemcpyDeviceToHost));
  if (fail) {
    char buf[320];
    snprintf(buf, sizeof buf,
             "prepare_temperatures: non-finite corrphotoionrenorm or bf-heating renormalisation in model cell %d "
             "(e.g. W = 0 or a zero analytic coefficient) -- the reference aborts here (update_grid.cc:911-918, "
             "959-965)",
             fail - 1);
    G.last_error = buf;
    return ARTIS_ERR_PACKET_FAULT;
  }
  HIPCHK(hipMemcpy(pr->TR_out, U.TR_out, npf * sizeof(float), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(pr->W_out, U.W_out, npf * sizeof(float), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(pr->TJ_out, U.TJ_out, npf * sizeof(float), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(pr->ffheating_out, U.ff_out, npf * sizeof(double), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(pr->colheating_out, U.col_out, npf * sizeof(double), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(pr->gamma_out, U.gam_out, npg * sizeof(double), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(pr->bfheating_out, U.bfh_out, npg * sizeof(double), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(pr->corrphotoionrenorm_out, U.renorm_out, npg * sizeof(double), hipMemcpyDeviceToHost));
  return 0;
}

}  // extern "C"

// ============================================================================== update_grid, nebular options
// artis_gpu_update_grid_nlte (include/artis_gpu.h, nlte_solver.h).  Host side: the atomic bookkeeping of the
// Spencer-Fano and rate-matrix layouts, the caller's arrays copied in, the kernels of solve_Te_nltepops per pass for
// the cells still iterating (the host reads back the convergence flags between passes), every array copied back on
// success.
namespace {
// nonthermal.cc:994-1007
double sf_get_J_host(int Z, int ionstage, double ionpot_ev) {
  if (ionstage == 1) {
    if (Z == 2) return 15.8;
    if (Z == 10) return 24.2;
    if (Z == 18) return 10.0;
  }
  return 0.6 * ionpot_ev;
}
// nonthermal.cc:1193-1309 get_mean_binding_energy; false on the reference's abort paths
bool sf_mean_binding_energy_host(const artis_nt_shells *nt, int Zel, int ioncharge, double ionpot, double *out) {
  const int nbound = Zel - ioncharge;
  double total = 0.0;
  if (nbound > 0) {
    int q[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
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
        else
          return false;
      } else if (ioncharge == 1) {
        if (q[9] < 1)
          q[9]++;
        else if (q[7] < 4)
          q[7]++;
        else if (q[8] < 6)
          q[8]++;
        else
          return false;
      } else if (ioncharge > 1) {
        if (q[7] < 4)
          q[7]++;
        else if (q[8] < 6)
          q[8]++;
        else
          return false;
      }
    }
    if (Zel < 1 || Zel > 30) return false;
    for (int electron_loop = 0; electron_loop < 10; electron_loop++) {
      const double electronsinshell = q[electron_loop];
      if (electronsinshell > 0) {
        double use2 = nt->electron_binding[(Zel - 1) * 10 + electron_loop];
        const double use3 = ionpot;
        if (use2 <= 0) {
          use2 = nt->electron_binding[(Zel - 1) * 10 + electron_loop - 1];
          if (electron_loop != 8) return false;
        }
        if (use2 < use3)
          total += electronsinshell / use3;
        else
          total += electronsinshell / use2;
      }
    }
  }
  *out = total;
  return true;
}
}  // namespace

extern "C" {
int artis_gpu_update_grid_nlte(const artis_nt_shells *nt, const artis_nlte_params *p, artis_nlte_cells *c) {
  if (!G.initialised) return ARTIS_ERR_NOT_INITIALISED;
  const DevRun &R = G.K.R;
  if (!R.nlte_on || !R.no_lut_photoion || !R.no_lut_bfheating || !R.multibin) {
    G.last_error = "update_grid_nlte: needs the nebular options (NLTE_POPS_ON, NO_LUT_PHOTOION / BFHEATING, MULTIBIN)";
    return ARTIS_ERR_UNSUPPORTED;
  }
  const bool sf_on = R.nt_on && R.nt_solve_spencerfano;
  if (R.nt_on && R.nt_max_auger != ARTIS_NT_MAX_AUGER) {
    G.last_error = "update_grid_nlte: nt_max_auger_electrons must be ARTIS_NT_MAX_AUGER";
    return ARTIS_ERR_UNSUPPORTED;
  }
  if (!p || !c || c->ncells < 0 || (c->ncells > 0 && !c->mgi) || !c->rho || !c->elem_abundance ||
      !c->elem_meanweight || !c->vol_init || !c->thick || !c->J || !c->nuJ || !c->ffheating || !c->bin_J_raw ||
      !c->bin_nuJ_raw || !c->bin_contribcount || !c->TR || !c->W || !c->TJ || !c->Te || !c->nne || !c->nnetot ||
      !c->groundlevelpop || !c->partfunct || !c->nlte_pops || !c->bin_TR || !c->bin_W || !c->totalcooling ||
      !c->cooling_contrib_ion || (R.detailed_bf && (!c->bfrate_raw || !c->bfrate_estimator)) ||
      (R.nt_on && (!c->deposition_rate_density || !c->nt_ionization_ratecoeff || !c->nt_eff_ionpot ||
                   !c->nt_frac_heating || !c->nt_frac_ionization || !c->nt_frac_excitation ||
                   !c->nt_nneperion_when_solved || !c->nt_timestep_last_solved || !c->nt_fracdep_ionization_ion ||
                   !c->nt_prob_num_auger || !c->nt_ionenfrac_num_auger)) ||
      (sf_on && (!nt || nt->sfpts < 2 || nt->sfpts > SF_NMAX || !(nt->sf_emax > nt->sf_emin) || nt->nshells < 0 ||
                 (nt->nshells > 0 && (!nt->Z || !nt->nelec || !nt->ionpot_ev || !nt->A || !nt->B || !nt->C ||
                                      !nt->D || !nt->prob_num_auger || !nt->en_auger_ev)) ||
                 !nt->electron_binding)) ||
      !(p->T_min > 0. && p->T_max > p->T_min && p->accuracy > 0. && p->tmin > 0. && p->t_current_te > 0. &&
        p->deltat > 0. && p->tratmid > 0. && p->nprocs > 0 && p->T_R_max > p->T_R_min && p->nlteiter >= 0)) {
    G.last_error = "update_grid_nlte: NULL array or bad parameters";
    return ARTIS_ERR_BAD_ARGUMENT;
  }
  const int np = G.npts_model, ne = G.nelements, ni = G.nions_total;
  const DevTab &T = G.K.T;
  const int nl = T.nlevels_total, nbf = T.nbf, nbins = T.rf_nbins, ntl = T.total_nlte_levels;
  const int64_t ntg = T.ntargets_total;
  for (int k = 0; k < c->ncells; k++)
    if (c->mgi[k] < 0 || c->mgi[k] >= np) {
      G.last_error = "update_grid_nlte: cell index out of range";
      return ARTIS_ERR_BAD_ARGUMENT;
    }
  if (c->ncells == 0) return 0;
  HIPCHK(hipEventRecord(G.ev2, G.stream));
  // host copies of the atomic bookkeeping the layouts need
  std::vector<int32_t> nions, uoff, ion_nlev, ion_ul0, ionis, nlte_n, nlte_first, ionstage, lev_nup, lev_upoff;
  std::vector<double> lev_eps;
  std::vector<float> lev_g;
  if (d2h_vec(nions, T.elem_nions, ne) || d2h_vec(uoff, T.elem_uniqueionoffset, ne) ||
      d2h_vec(ion_nlev, T.ion_nlevels, ni) || d2h_vec(ion_ul0, T.ion_uniqueleveloffset, ni) ||
      d2h_vec(ionis, T.ion_ionisinglevels, ni) || d2h_vec(nlte_n, T.ion_nlevels_nlte, ni) ||
      d2h_vec(nlte_first, T.ion_first_nlte, ni) || d2h_vec(ionstage, T.ion_ionstage, ni) ||
      d2h_vec(lev_nup, T.level_nuptrans, nl) || d2h_vec(lev_upoff, T.level_uptrans_offset, nl) ||
      d2h_vec(lev_eps, T.level_epsilon, nl) || d2h_vec(lev_g, T.level_stat_weight, nl))
    return ARTIS_ERR_HIP;
  // calculate_heating_rates' bf-heating levels (thermalbalance.cc:304-310)
  std::vector<int32_t> hb;
  for (int e = 0; e < ne; e++) {
    if (nions[e] > TE_MAX_IONS_PER_ELEMENT) {
      G.last_error = "update_grid_nlte: more ions per element than TE_MAX_IONS_PER_ELEMENT";
      return ARTIS_ERR_UNSUPPORTED;
    }
    for (int i = 0; i < nions[e] - 1; i++)
      for (int l = 0; l < ionis[uoff[e] + i]; l++) hb.push_back(ion_ul0[uoff[e] + i] + l);
  }
  // the LTE-branch and the iterated cells
  std::vector<int32_t> lte_list, nl_list;
  for (int k = 0; k < c->ncells; k++) {
    const int mgi = c->mgi[k];
    if (p->initial_iteration || c->thick[mgi] == 1)
      lte_list.push_back(mgi);
    else
      nl_list.push_back(mgi);
  }
  const int nnl = (int)nl_list.size();
  const size_t npf = np, npi = (size_t)np * ni, npe = (size_t)np * ne, A1 = NL_A1;
  DevBufs B;
  NlDev N{};
  int rc = 0;
  N.np = np;
  N.ncells = c->ncells;
  rc |= B.get((int32_t **)&N.mgi, (size_t)c->ncells, c->mgi);
  N.nts = p->nts;
  N.num_lte_timesteps = p->num_lte_timesteps;
  N.initial_iteration = p->initial_iteration;
  N.nprocs = p->nprocs;
  N.do_rlc_est = p->do_rlc_est;
  N.nt_on = R.nt_on;
  N.sf_on = sf_on;
  N.deltat = p->deltat;
  N.tratmid = p->tratmid;
  N.T_min = p->T_min;
  N.T_max = p->T_max;
  N.T_R_min = p->T_R_min;
  N.T_R_max = p->T_R_max;
  rc |= B.get((float **)&N.rho, npf, c->rho);
  rc |= B.get((float **)&N.abund, npe, c->elem_abundance);
  rc |= B.get((float **)&N.meanw, npe, c->elem_meanweight);
  rc |= B.get((double **)&N.vol, npf, c->vol_init);
  rc |= B.get((int16_t **)&N.thick, npf, c->thick);
  rc |= B.get((double **)&N.dep, npf, R.nt_on ? c->deposition_rate_density : nullptr);
  rc |= B.get((double **)&N.J, npf, c->J);
  rc |= B.get((double **)&N.nuJ, npf, c->nuJ);
  rc |= B.get((double **)&N.ffraw, npf, c->ffheating);
  rc |= B.get((double **)&N.bfraw, (size_t)np * nbf, R.detailed_bf ? c->bfrate_raw : nullptr);
  rc |= B.get((double **)&N.binJ, (size_t)np * nbins, c->bin_J_raw);
  rc |= B.get((double **)&N.binnuJ, (size_t)np * nbins, c->bin_nuJ_raw);
  rc |= B.get((int64_t **)&N.bincount, (size_t)np * nbins, c->bin_contribcount);
  rc |= B.get(&N.TR, npf, c->TR);
  rc |= B.get(&N.W, npf, c->W);
  rc |= B.get(&N.TJ, npf, c->TJ);
  rc |= B.get(&N.Te, npf, c->Te);
  rc |= B.get(&N.nne, npf, c->nne);
  rc |= B.get(&N.nnetot, npf, c->nnetot);
  rc |= B.get(&N.gp, npi, c->groundlevelpop);
  rc |= B.get(&N.pf, npi, c->partfunct);
  rc |= B.get(&N.nlte, (size_t)np * std::max(1, ntl), c->nlte_pops);
  rc |= B.get(&N.binTR, (size_t)np * nbins, c->bin_TR);
  rc |= B.get(&N.binW, (size_t)np * nbins, c->bin_W);
  rc |= B.get(&N.bfrate, (size_t)np * std::max(1, nbf), R.detailed_bf ? c->bfrate_estimator : nullptr);
  if (R.nt_on) {
    rc |= B.get(&N.nt_fh, npf, c->nt_frac_heating);
    rc |= B.get(&N.nt_fi, npf, c->nt_frac_ionization);
    rc |= B.get(&N.nt_fe, npf, c->nt_frac_excitation);
    rc |= B.get(&N.nt_nneper, npf, c->nt_nneperion_when_solved);
    rc |= B.get(&N.nt_tls, npf, c->nt_timestep_last_solved);
    rc |= B.get(&N.nt_effion, npi, c->nt_eff_ionpot);
    rc |= B.get(&N.nt_fracdep, npi, c->nt_fracdep_ionization_ion);
    rc |= B.get(&N.nt_prob, npi * A1, c->nt_prob_num_auger);
    rc |= B.get(&N.nt_ionen, npi * A1, c->nt_ionenfrac_num_auger);
    rc |= B.get(&N.ntY, npi, (const double *)nullptr);
  }
  rc |= B.get(&N.ffheat, npf, (const double *)nullptr);
  rc |= B.get(&N.hdep, npf, (const double *)nullptr);
  rc |= B.get(&N.prevTe, npf, (const double *)nullptr);
  rc |= B.get(&N.fail, 2, (const int32_t *)nullptr);
  double *d_totcool = nullptr, *d_ccion = nullptr, *d_rates = nullptr;
  rc |= B.get(&d_totcool, npf, c->totalcooling);
  rc |= B.get(&d_ccion, npi, c->cooling_contrib_ion);
  rc |= B.get(&d_rates, npf * ARTIS_TE_NRATES, (const double *)c->heatingcoolingrates);
  if (rc) return ARTIS_ERR_HIP;
  if (R.nt_on) HIPCHK(hipMemcpyAsync(N.ntY, c->nt_ionization_ratecoeff, npi * sizeof(double), hipMemcpyHostToDevice, G.stream));
  if (!c->heatingcoolingrates) HIPCHK(hipMemsetAsync(d_rates, 0, npf * ARTIS_TE_NRATES * sizeof(double), G.stream));
  HIPCHK(hipMemsetAsync(N.fail, 0, 2 * sizeof(int32_t), G.stream));
  HIPCHK(hipMemsetAsync(N.ffheat, 0, npf * sizeof(double), G.stream));
  HIPCHK(hipMemsetAsync(N.hdep, 0, npf * sizeof(double), G.stream));
  // the solver's context: the cell-state pointers at the solver's arrays, the active cells as the "non-empty" list
  Ctx KN = G.K;
  KN.R.nts = p->nts;
  KN.C.Te = N.Te;
  KN.C.TR = N.TR;
  KN.C.TJ = N.TJ;
  KN.C.W = N.W;
  KN.C.nne = N.nne;
  KN.C.nnetot = N.nnetot;
  KN.C.rho = N.rho;
  KN.C.thick = N.thick;
  KN.C.elem_abundance = N.abund;
  KN.C.groundlevelpop = N.gp;
  KN.C.partfunct = N.pf;
  KN.C.nlte_pops = N.nlte;
  KN.C.rf_TR = N.binTR;
  KN.C.rf_W = N.binW;
  KN.C.bfrate_est = N.bfrate;
  KN.C.nt_dep = N.dep;
  KN.C.nt_Y = N.ntY;
  KN.C.nt_prob = N.nt_prob;
  KN.C.nt_ionen = N.nt_ionen;
  const int nact_max = std::max(1, nnl);
  int32_t *d_act = nullptr, *d_actk = nullptr, *d_lte = nullptr, *d_nl = nullptr;
  double *d_pops = nullptr, *d_corr = nullptr, *d_hbc = nullptr;
  double2 *d_depr = nullptr;
  rc |= B.get(&d_act, (size_t)nact_max, (const int32_t *)nullptr);
  rc |= B.get(&d_actk, (size_t)nact_max, (const int32_t *)nullptr);
  rc |= B.get(&d_lte, std::max<size_t>(1, lte_list.size()), lte_list.empty() ? nullptr : lte_list.data());
  rc |= B.get(&d_nl, (size_t)nact_max, nl_list.empty() ? nullptr : nl_list.data());
  rc |= B.get(&d_pops, (size_t)nact_max * nl, (const double *)nullptr);
  rc |= B.get(&d_corr, (size_t)nact_max * (ntg + 1), (const double *)nullptr);
  rc |= B.get(&d_depr, (size_t)nact_max * std::max(1, nbf), (const double2 *)nullptr);
  rc |= B.get(&d_hbc, std::max<size_t>(1, hb.size()) * nact_max, (const double *)nullptr);
  if (rc) return ARTIS_ERR_HIP;
  KN.C.pops = d_pops;
  KN.C.corrphot = d_corr;
  KN.C.bfcell = d_depr;
  KN.C.ionpop = nullptr;  // (k_bfcells writes only the departure ratios here)
  KN.C.ne_mgi = d_act;
  KN.C.n_nonempty = 0;
  KN.C.linecoef = nullptr;
  KN.C.linecoef_rows = 0;
  // the thermal-balance solver's view (te_solver.h) of the same state
  TeDev D{};
  rc |= B.get((int32_t **)&D.anumber, (size_t)ne, G.h_anumber.data());
  rc |= B.get((int32_t **)&D.hb_ul, std::max<size_t>(1, hb.size()), hb.empty() ? nullptr : hb.data());
  rc |= B.get(&D.upp, npe, (const int32_t *)nullptr);
  if (rc) return ARTIS_ERR_HIP;
  D.nhb = (int32_t)hb.size();
  D.t_current = p->t_current_te;
  D.tmin = p->tmin;
  D.T_min = p->T_min;
  D.T_max = p->T_max;
  D.accuracy = p->accuracy;
  D.initial_iteration = p->initial_iteration;
  D.TR = N.TR;
  D.W = N.W;
  D.TJ = N.TJ;
  D.rho = N.rho;
  D.abund = N.abund;
  D.meanw = N.meanw;
  D.thick = N.thick;
  D.vol = N.vol;
  D.ffheat = N.ffheat;
  D.hdep = N.hdep;
  D.Te = N.Te;
  D.gp = N.gp;
  D.nne = N.nne;
  D.nnetot = N.nnetot;
  D.pf = N.pf;
  D.totcool = d_totcool;
  D.ccion = d_ccion;
  D.rates = d_rates;
  D.hbc = d_hbc;
  D.fail = N.fail;
  D.direct_col_heat = 1;
  D.nlte = N.nlte;
  D.hbstride = nact_max;
  Ctx *dK = nullptr;
  TeDev *dD = nullptr;
  NlDev *dN = nullptr;
  if (B.get(&dK, 1, &KN) || B.get(&dD, 1, (const TeDev *)nullptr) || B.get(&dN, 1, &N)) return ARTIS_ERR_HIP;
  const int g = te_lanes_per_cell(ni);
  const int cpw = 64 / g;
  auto te_launch = [&](const int32_t *list, int n, int mode, const int32_t *hbk) -> int {
    if (n <= 0) return 0;
    D.mgi = list;
    D.ncells = n;
    D.mode = mode;
    D.hbk = hbk;
    HIPCHK(hipStreamSynchronize(G.stream));  // dD is read by the previous launch
    HIPCHK(hipMemcpy(dD, &D, sizeof(TeDev), hipMemcpyHostToDevice));
    k_te_solve<<<(unsigned)((n + cpw - 1) / cpw), 64, (size_t)cpw * ni * sizeof(double), G.stream>>>(dK, dD, g);
    HIPCHK(hipGetLastError());
    return 0;
  };
  auto read_fail = [&](const char *where) -> int {
    int32_t f[2] = {0, 0};
    HIPCHK(hipStreamSynchronize(G.stream));
    HIPCHK(hipMemcpy(f, N.fail, sizeof f, hipMemcpyDeviceToHost));
    if (!f[0]) return 0;
    static const char *why[] = {"a GSL root-finder error of call_T_e_finder / calculate_populations",
                                "a GSL root-finder error of the radiation-field bin fit (find_T_R)",
                                "a non-finite bf-heating coefficient",
                                "get_mean_binding_energy has no shell data for the work-function approximation",
                                "non-finite or negative NLTE populations", "the T_e finder"};
    char buf[320];
    snprintf(buf, sizeof buf, "update_grid_nlte (%s): %s in model cell %d -- the reference aborts here", where,
             why[(f[1] >= 0 && f[1] <= 5) ? f[1] : 0], f[0] - 1);
    G.last_error = buf;
    return ARTIS_ERR_PACKET_FAULT;
  };
  // ARTIS_GPU_NL_DEBUG=1: synchronise after every step and name the first one that fails
  const bool nl_debug = getenv("ARTIS_GPU_NL_DEBUG") && getenv("ARTIS_GPU_NL_DEBUG")[0] == '1';
  auto step = [&](const char *what) -> int {
    hipError_t e = hipGetLastError();
    if (e == hipSuccess && nl_debug) e = hipStreamSynchronize(G.stream);
    if (e != hipSuccess) {
      G.last_error = std::string("update_grid_nlte: ") + what + ": " + hipGetErrorString(e);
      return ARTIS_ERR_HIP;
    }
    return 0;
  };
#define NLSTEP(what)                  \
  do {                                \
    if (int e_ = step(what)) return e_; \
  } while (0)
  NLSTEP("uploads");
  const int TB = 256;
  k_nl_prepare<<<(c->ncells + TB - 1) / TB, TB, 0, G.stream>>>(N);
  NLSTEP("k_nl_prepare");
  // LTE-branch cells: precalculate_partfuncts + calculate_populations (LTE phi) + the cooling rates
  if (int e2 = te_launch(d_lte, (int)lte_list.size(), 0, nullptr)) return e2;
  NLSTEP("k_te_solve (LTE branch)");
  // Spencer-Fano tables
  SfDev S{};
  std::vector<int32_t> h_solve;
  int sf_batch = 1;
  std::vector<double> h_none;  // errbest seeds (-1: no solution yet)
  if (sf_on && nnl > 0) {
    const int n = nt->sfpts;
    S.n = n;
    S.emin = nt->sf_emin;
    S.emax = nt->sf_emax;
    S.DE = (S.emax - S.emin) / (n - 1);
    std::vector<double> envec(n), logenvec(n), sourcevec(n), pw2(n), rhs(n, 0.);
    const int source_spread_pts = (int)ceil(n * 0.03333);
    const double source_spread_en = source_spread_pts * S.DE;
    const int sourcelowerindex = n - source_spread_pts;
    for (int k = 0; k < n; k++) {
      envec[k] = S.emin + k * S.DE;
      logenvec[k] = log(envec[k]);
      sourcevec[k] = (k < sourcelowerindex) ? 0. : 1. / source_spread_en;
      pw2[k] = pow(envec[k] * ARTIS_EV, -2);
    }
    double E = 0.;
    for (int k = 0; k < n; k++) E += fabs((sourcevec[k] * S.DE) * envec[k]);
    S.E_init_ev = E;
    for (int i = 0; i < n - 1; i++) {
      double dasum = 0.;
      for (int j = i + 1; j < n; j++) dasum += fabs(sourcevec[j]);
      rhs[i] = dasum * S.DE;
    }
    auto gteq = [&](double en) {
      const int index = (int)ceil((en - S.emin) / S.DE);
      return index < 0 ? 0 : (index > n - 1 ? n - 1 : index);
    };
    // shells (collion.txt entries of each ion) and their tables
    std::vector<int32_t> sh_off(ni + 1, 0), sh_k, sh_start, sh_astop;
    std::vector<double> sh_ip, sh_J, sh_xs, sh_ieu, sh_atn, sh_ie2, sh_prob;
    std::vector<int32_t> tr_off(ni + 1, 0), tr_ul, tr_kind, tr_start, tr_build;
    std::vector<double> tr_cf, tr_logeps, tr_eps_ev, tr_eps, binding(ni, 0.);
    std::vector<int32_t> binding_ok(ni, 0);
    std::vector<int32_t> line_upper;
    std::vector<float> line_coll, line_f;
    std::vector<uint8_t> line_forb;
    std::vector<int32_t> upidx;
    const int64_t nup = lev_upoff.empty() ? 0 : (int64_t)lev_upoff[nl - 1] + lev_nup[nl - 1];
    if (d2h_vec(line_upper, T.line_upper, T.nlines) || d2h_vec(line_coll, T.line_coll, T.nlines) ||
        d2h_vec(line_f, T.line_f, T.nlines) || d2h_vec(line_forb, T.line_forbidden, T.nlines) ||
        d2h_vec(upidx, T.uptrans_lineindex, (size_t)std::max<int64_t>(nup, 0)))
      return ARTIS_ERR_HIP;
    int band = 1;
    for (int e = 0; e < ne; e++)
      for (int i = 0; i < nions[e]; i++) {
        const int u = uoff[e] + i;
        const int Z = G.h_anumber[e];
        const int ist = ionstage[u];
        for (int k = 0; k < nt->nshells; k++) {
          if (!(nt->Z[k] == Z && nt->nelec[k] == Z - ist + 1)) continue;
          const double ionpot_ev = nt->ionpot_ev[k];
          const double J = sf_get_J_host(Z, ist, ionpot_ev);
          const int xsstart = gteq(ionpot_ev);
          sh_k.push_back(k);
          sh_ip.push_back(ionpot_ev);
          sh_J.push_back(J);
          sh_start.push_back(xsstart);
          sh_astop.push_back(gteq((double)nt->en_auger_ev[k]));
          for (int q = 0; q < NL_A1; q++) sh_prob.push_back(nt->prob_num_auger[k * NL_A1 + q]);
          const double A = nt->A[k], Bc = nt->B[k], Cc = nt->C[k], Dc = nt->D[k];
          for (int j = 0; j < n; j++) {  // nonthermal.cc:952-976, 2370-2380
            double xs = 0., ieu = 0., atn = 0.;
            if (j >= xsstart) {
              const double uu = envec[j] / ionpot_ev;
              xs = 1e-14 * (A * (1 - 1 / uu) + Bc * pow((1 - 1 / uu), 2) + Cc * log(uu) + Dc * log(uu) / uu) /
                   (uu * pow(ionpot_ev, 2));
              const double endash = envec[j];
              const double epsilon_upper = std::min((endash + ionpot_ev) / 2, endash);
              ieu = atan((epsilon_upper - ionpot_ev) / J);
              atn = atan((endash - ionpot_ev) / 2 / J);
            }
            sh_xs.push_back(xs);
            sh_ieu.push_back(ieu);
            sh_atn.push_back(atn);
            sh_ie2.push_back(atan(envec[j] / J));
          }
        }
        sh_off[u + 1] = (int32_t)sh_k.size();
        // excitation transitions (nonthermal.cc:2282-2341, 872-929)
        const int nlev5 = std::min(ion_nlev[u], 5);
        for (int lower = 0; lower < nlev5; lower++) {
          const int ul = ion_ul0[u] + lower;
          const double statweight_lower = lev_g[ul];
          for (int t = 0; t < lev_nup[ul]; t++) {
            const int li = upidx[lev_upoff[ul] + t];
            const int upper = line_upper[li];
            if (upper >= 250) continue;
            const double epsilon_trans = lev_eps[ion_ul0[u] + upper] - lev_eps[ul];
            const double eps_ev = epsilon_trans / ARTIS_EV;
            const double coll_str = line_coll[li];
            int kind;
            double cf, logeps = 0.;
            if (coll_str >= 0) {
              kind = 0;
              cf = pow(ARTIS_H_IONPOT, 2) / statweight_lower * coll_str * ARTIS_PI * 2.800285203e-17;
            } else if (!line_forb[li]) {
              kind = 1;
              const double fij = line_f[li];
              cf = eps_ev * 45.585750051 * 2.800285203e-17 * pow(ARTIS_H_IONPOT / epsilon_trans, 2) * fij;
              logeps = log(eps_ev);
            } else {
              continue;
            }
            tr_ul.push_back(ul);
            tr_kind.push_back(kind);
            tr_start.push_back(gteq(eps_ev));
            tr_build.push_back(!(eps_ev < S.emin));
            tr_cf.push_back(cf);
            tr_logeps.push_back(logeps);
            tr_eps_ev.push_back(eps_ev);
            tr_eps.push_back(epsilon_trans);
            if (!(eps_ev < S.emin)) band = std::max(band, (int)ceil(eps_ev / S.DE) + 2);
          }
        }
        tr_off[u + 1] = (int32_t)tr_ul.size();
        double bnd = 0.;
        binding_ok[u] = sf_mean_binding_energy_host(nt, Z, ist - 1, G.h_ion_ionpot[u], &bnd) ? 1 : 0;
        binding[u] = bnd;
      }
    S.band = band;
    S.nsh = (int32_t)sh_k.size();
    S.nitems = S.nsh + (int32_t)tr_ul.size();
    auto up = [&](auto **d, const auto &v) {
      using Tv = typename std::remove_reference<decltype(v)>::type::value_type;
      return B.get((Tv **)d, std::max<size_t>(1, v.size()), v.empty() ? nullptr : v.data());
    };
    rc |= up(&S.envec, envec);
    rc |= up(&S.logenvec, logenvec);
    rc |= up(&S.pw2, pw2);
    rc |= up(&S.rhs, rhs);
    rc |= up(&S.ion_sh_off, sh_off);
    rc |= up(&S.sh_k, sh_k);
    rc |= up(&S.sh_xsstart, sh_start);
    rc |= up(&S.sh_augerstop, sh_astop);
    rc |= up(&S.sh_ionpot_ev, sh_ip);
    rc |= up(&S.sh_J, sh_J);
    rc |= up(&S.sh_xs, sh_xs);
    rc |= up(&S.sh_ieu, sh_ieu);
    rc |= up(&S.sh_atn, sh_atn);
    rc |= up(&S.sh_ie2, sh_ie2);
    rc |= up(&S.sh_prob, sh_prob);
    rc |= up(&S.ion_tr_off, tr_off);
    rc |= up(&S.tr_ul, tr_ul);
    rc |= up(&S.tr_kind, tr_kind);
    rc |= up(&S.tr_start, tr_start);
    rc |= up(&S.tr_build, tr_build);
    rc |= up(&S.tr_cf, tr_cf);
    rc |= up(&S.tr_logeps, tr_logeps);
    rc |= up(&S.tr_eps_ev, tr_eps_ev);
    rc |= up(&S.tr_eps, tr_eps);
    rc |= up(&S.ion_binding, binding);
    rc |= up(&S.ion_binding_ok, binding_ok);
    S.anumber = D.anumber;
    // cells solved together: their matrices (8 n^2 bytes each) within ARTIS_GPU_SF_BATCH_GB (default 8 GiB)
    double sf_gb = 8.;
    if (const char *v = getenv("ARTIS_GPU_SF_BATCH_GB")) sf_gb = std::max(0.0, atof(v));
    sf_batch = (int)std::max<double>(1., std::min<double>(nnl, sf_gb * (double)(1ull << 30) / (8.0 * n * n)));
    h_none.assign(sf_batch, -1.);
    const size_t nbq = (size_t)sf_batch;
    rc |= B.get((int32_t **)&S.bat_a, nbq, (const int32_t *)nullptr);
    rc |= B.get((int32_t **)&S.bat_mgi, nbq, (const int32_t *)nullptr);
    rc |= B.get(&S.nnion, nbq * ni, (const double *)nullptr);
    rc |= B.get(&S.incl, nbq * ni, (const int32_t *)nullptr);
    rc |= B.get(&S.tot_nion, nbq, (const double *)nullptr);
    rc |= B.get(&S.MT, nbq * n * n, (const double *)nullptr);
    rc |= B.get(&S.x, nbq * n, (const double *)nullptr);
    rc |= B.get(&S.best, nbq * n, (const double *)nullptr);
    rc |= B.get(&S.work, nbq * n, (const double *)nullptr);
    rc |= B.get(&S.res, nbq * n, (const double *)nullptr);
    rc |= B.get(&S.part, nbq * n * ((n + SF_RCHUNK - 1) / SF_RCHUNK), (const double *)nullptr);
    rc |= B.get(&S.errbest, nbq, (const double *)nullptr);
    rc |= B.get(&S.dots, nbq * std::max(1, S.nitems), (const double *)nullptr);
    rc |= B.get(&S.solve, (size_t)nact_max, (const int32_t *)nullptr);
    if (rc) return ARTIS_ERR_HIP;
  } else if (R.nt_on) {
    // the binding energies the work-function fallback of nt_ionization_ratecoeff reads
    std::vector<double> binding(ni, 0.);
    std::vector<int32_t> binding_ok(ni, 0);
    if (nt && nt->electron_binding)
      for (int e = 0; e < ne; e++)
        for (int i = 0; i < nions[e]; i++) {
          const int u = uoff[e] + i;
          double bnd = 0.;
          binding_ok[u] = sf_mean_binding_energy_host(nt, G.h_anumber[e], ionstage[u] - 1, G.h_ion_ionpot[u], &bnd);
          binding[u] = bnd;
        }
    rc |= B.get((double **)&S.ion_binding, (size_t)ni, binding.data());
    rc |= B.get((int32_t **)&S.ion_binding_ok, (size_t)ni, binding_ok.data());
    S.anumber = D.anumber;
    if (rc) return ARTIS_ERR_HIP;
  }
  // the rate-matrix layout: per element D = sum over ions of nlevels_nlte + 1 (+ 1 with a superlevel)
  NlMat M{};
  std::vector<int32_t> el_D(ne, 0), el_off1(ne, 0), col_e, col_ion, col_l0, col_l1;
  std::vector<int64_t> el_off2(ne, 0);
  int64_t cell2 = 0;
  int cell1 = 0;
  for (int e = 0; e < ne; e++) {
    el_off1[e] = cell1;
    el_off2[e] = cell2;
    int Dm = 0;
    for (int i = 0; i < nions[e]; i++) {
      const int u = uoff[e] + i;
      const int nn = nlte_n[u];
      for (int l = 0; l <= nn && l < ion_nlev[u]; l++) {
        col_e.push_back(e);
        col_ion.push_back(i);
        col_l0.push_back(l);
        col_l1.push_back(l);
      }
      Dm += nn + 1;
      if (ion_nlev[u] > nn + 1) {
        col_e.push_back(e);
        col_ion.push_back(i);
        col_l0.push_back(nn + 1);
        col_l1.push_back(ion_nlev[u] - 1);
        Dm += 1;
      }
    }
    el_D[e] = Dm;
    cell1 += Dm;
    cell2 += (int64_t)Dm * Dm;
  }
  if ((int)col_e.size() != cell1) {
    G.last_error = "update_grid_nlte: an ion with fewer levels than nlevels_nlte + 1";
    return ARTIS_ERR_UNSUPPORTED;
  }
  M.cell1 = cell1;
  M.cell2 = cell2;
  M.t_mid = p->t_mid;
  const double per_cell = (7.0 * cell2 + 8.0 * cell1) * 8.0 + 4.0 * (cell1 + ne);
  const int chunk = std::max(1, std::min(nact_max, (int)std::min(1e9, (double)(1ll << 30) / per_cell)));
  rc |= B.get((int32_t **)&M.el_D, (size_t)ne, el_D.data());
  rc |= B.get((int32_t **)&M.el_off1, (size_t)ne, el_off1.data());
  rc |= B.get((int64_t **)&M.el_off2, (size_t)ne, el_off2.data());
  rc |= B.get((int32_t **)&M.col_e, std::max<size_t>(1, col_e.size()), col_e.data());
  rc |= B.get((int32_t **)&M.col_ion, std::max<size_t>(1, col_ion.size()), col_ion.data());
  rc |= B.get((int32_t **)&M.col_l0, std::max<size_t>(1, col_l0.size()), col_l0.data());
  rc |= B.get((int32_t **)&M.col_l1, std::max<size_t>(1, col_l1.size()), col_l1.data());
  rc |= B.get(&M.A, (size_t)chunk * std::max<int64_t>(1, cell2), (const double *)nullptr);
  rc |= B.get(&M.LU, (size_t)chunk * std::max<int64_t>(1, cell2), (const double *)nullptr);
  rc |= B.get(&M.P, (size_t)chunk * 5 * std::max<int64_t>(1, cell2), (const double *)nullptr);
  for (double **v : {&M.b, &M.norm, &M.pv, &M.xv, &M.best, &M.work, &M.res})
    rc |= B.get(v, (size_t)chunk * std::max(1, cell1), (const double *)nullptr);
  rc |= B.get(&M.perm, (size_t)chunk * std::max(1, cell1), (const int32_t *)nullptr);
  rc |= B.get(&M.status, (size_t)chunk * ne, (const int32_t *)nullptr);
  rc |= B.get(&M.slpf, (size_t)nact_max * ni, (const double *)nullptr);
  rc |= B.get(&M.done, (size_t)nact_max, (const int32_t *)nullptr);
  // the integration workspace (the engine's, or one of its own)
  QagWs ws = G.qag;
  int qwaves = G.qag_waves;
  if (qwaves <= 0) {
    qwaves = 64;
    const size_t nw = (size_t)qwaves * QAG_LIMIT;
    rc |= B.get(&ws.alist, nw, (const double *)nullptr);
    rc |= B.get(&ws.blist, nw, (const double *)nullptr);
    rc |= B.get(&ws.rlist, nw, (const double *)nullptr);
    rc |= B.get(&ws.elist, nw, (const double *)nullptr);
    rc |= B.get(&ws.order, nw, (const int32_t *)nullptr);
    rc |= B.get(&ws.level, nw, (const int32_t *)nullptr);
  }
  if (rc) return ARTIS_ERR_HIP;
  std::vector<int32_t> h_iters(c->ncells, 0);
  if (nnl > 0) {
    // radiation-field fit and bf-heating coefficients of the iterated cells
    if (nbf > 0 && R.detailed_bf)
      k_nl_bfnorm<<<(unsigned)(((int64_t)nnl * nbf + TB - 1) / TB), TB, 0, G.stream>>>(KN, N, d_nl, nnl);
    NLSTEP("k_nl_bfnorm");
    if (nbins > 0)
      k_nl_binfit<<<(unsigned)(((int64_t)nnl * nbins + 63) / 64), 64, 0, G.stream>>>(dK, dN, d_nl, nnl);
    NLSTEP("k_nl_binfit");
    if (!hb.empty())
      k_nl_bfheat<<<(unsigned)std::min<int64_t>((int64_t)nnl * hb.size(), qwaves), 64, 0, G.stream>>>(
          dK, dN, d_nl, nnl, D.hb_ul, (int)hb.size(), d_hbc, ws);
    NLSTEP("k_nl_bfheat");
    if (int e2 = read_fail("radiation field / bf heating")) return e2;
    D.hbstride = nnl;
    // solve_Te_nltepops passes for the cells still iterating
    std::vector<int32_t> act = nl_list, actk(nnl);
    for (int k = 0; k < nnl; k++) actk[k] = k;
    std::map<int, int> k_of_mgi;
    for (int k = 0; k < c->ncells; k++) k_of_mgi[c->mgi[k]] = k;
    for (int iter = 0; iter <= p->nlteiter && !act.empty(); iter++) {
      const int nact = (int)act.size();
      HIPCHK(hipMemcpyAsync(d_act, act.data(), nact * sizeof(int32_t), hipMemcpyHostToDevice, G.stream));
      HIPCHK(hipMemcpyAsync(d_actk, actk.data(), nact * sizeof(int32_t), hipMemcpyHostToDevice, G.stream));
      KN.C.n_nonempty = nact;
      const int64_t nlv = (int64_t)nact * nl;
      if (sf_on) {
        k_levelpops<<<(unsigned)((nlv + TB - 1) / TB), TB, 0, G.stream>>>(KN);
        NLSTEP("k_levelpops (Spencer-Fano)");
        k_sf_decide<<<(nact + TB - 1) / TB, TB, 0, G.stream>>>(KN, N, S, d_act, nact);
        NLSTEP("k_sf_decide");
        HIPCHK(hipStreamSynchronize(G.stream));
        if (d2h_vec(h_solve, S.solve, nact)) return ARTIS_ERR_HIP;
        const int n = S.n;
        std::vector<int32_t> sa, sm;  // the cells to solve: active position, model cell
        for (int a = 0; a < nact; a++)
          if (h_solve[a]) {
            sa.push_back(a);
            sm.push_back(act[a]);
          }
        for (size_t q0 = 0; q0 < sa.size(); q0 += sf_batch) {
          const int nb = (int)std::min<size_t>(sf_batch, sa.size() - q0);
          HIPCHK(hipMemcpy((void *)S.bat_a, sa.data() + q0, nb * sizeof(int32_t), hipMemcpyHostToDevice));
          HIPCHK(hipMemcpy((void *)S.bat_mgi, sm.data() + q0, nb * sizeof(int32_t), hipMemcpyHostToDevice));
          k_sf_ions<<<(nb * ni + 63) / 64, 64, 0, G.stream>>>(KN, N, S, nb);
          NLSTEP("k_sf_ions");
          k_sf_matrix<<<dim3((unsigned)((n + 255) / 256), (unsigned)n, (unsigned)nb), 256, 0, G.stream>>>(KN, N, S,
                                                                                                         d_pops);
          NLSTEP("k_sf_matrix");
          for (int q = 0; q < nb; q++)
            HIPCHK(hipMemcpyAsync(S.x + (size_t)q * n, S.rhs, n * sizeof(double), hipMemcpyDeviceToDevice, G.stream));
          k_sf_backsub<<<nb, SF_WG, 0, G.stream>>>(S.MT, n, S.x);
          NLSTEP("k_sf_backsub");
          HIPCHK(hipMemcpyAsync(S.errbest, h_none.data(), nb * sizeof(double), hipMemcpyHostToDevice, G.stream));
          const dim3 rgrid((unsigned)((n + 255) / 256), (unsigned)((n + SF_RCHUNK - 1) / SF_RCHUNK), (unsigned)nb);
          const dim3 vgrid((unsigned)((n + 255) / 256), (unsigned)nb);
          for (int it = 0; it < 10; it++) {
            if (it > 0) {
              k_sf_residual_part<<<rgrid, 256, 0, G.stream>>>(S.MT, n, S.x, S.part);
              k_sf_residual_sum<<<vgrid, 256, 0, G.stream>>>(n, S.part, S.rhs, S.work);
              k_sf_backsub<<<nb, SF_WG, 0, G.stream>>>(S.MT, n, S.work);
              k_sf_axpy<<<vgrid, 256, 0, G.stream>>>(n, S.x, S.work);
            }
            k_sf_residual_part<<<rgrid, 256, 0, G.stream>>>(S.MT, n, S.x, S.part);
            k_sf_residual_sum<<<vgrid, 256, 0, G.stream>>>(n, S.part, S.rhs, S.res);
            k_sf_best<<<nb, 1024, 0, G.stream>>>(n, S.res, S.x, S.best, S.errbest);
            NLSTEP("Spencer-Fano refinement");
          }
          k_sf_dots<<<dim3((unsigned)((S.nitems + 63) / 64), (unsigned)nb), 64, 0, G.stream>>>(S, S.best);
          NLSTEP("k_sf_dots");
          k_sf_combine<<<(nb + 63) / 64, 64, 0, G.stream>>>(KN, N, S, d_pops, nb);
          NLSTEP("k_sf_combine");
          HIPCHK(hipStreamSynchronize(G.stream));  // the batch lists and errbest seeds are reused
        }
      }
      k_nl_ntrates<<<(nact + TB - 1) / TB, TB, 0, G.stream>>>(KN, N, S, d_act, nact);
      NLSTEP("k_nl_ntrates");
      if (int e2 = te_launch(d_act, nact, 1, d_actk)) return e2;
      NLSTEP("k_te_solve (call_T_e_finder)");
      if (int e2 = read_fail("call_T_e_finder")) return e2;
      // populations and corrected photoionisation coefficients at the new T_e; the rate matrices
      k_levelpops<<<(unsigned)((nlv + TB - 1) / TB), TB, 0, G.stream>>>(KN);
      NLSTEP("k_levelpops");
      const int64_t nbt = (int64_t)nact * (nbf + ntg);
      if (nbt > 0) k_bfcells<<<(unsigned)((nbt + TB - 1) / TB), TB, 0, G.stream>>>(KN, G.d_target_ul, G.d_target_t);
      NLSTEP("k_bfcells");
      if (ntg > 0)
        k_corrphot_integral<<<(unsigned)std::min<int64_t>((int64_t)nact * ntg, qwaves), 64, 0, G.stream>>>(
            KN, G.d_target_ul, G.d_target_t, ws);
      NLSTEP("k_corrphot_integral");
      k_nl_slpf<<<(unsigned)(((int64_t)nact * ni + TB - 1) / TB), TB, 0, G.stream>>>(KN, N, M, d_act, nact);
      NLSTEP("k_nl_slpf");
      for (int a0 = 0; a0 < nact; a0 += chunk) {
        const int nch = std::min(chunk, nact - a0);
        if (cell1 > 0) {
          k_nl_matrix<<<(unsigned)(((int64_t)nch * cell1 + 63) / 64), 64, 0, G.stream>>>(KN, N, M, d_act, a0, nch);
          NLSTEP("k_nl_matrix");
          k_nl_lu<<<(unsigned)(nch * ne), NL_LU_WG, 0, G.stream>>>(KN, M, nch);
          NLSTEP("k_nl_lu");
          if (a0 == 0 && getenv("ARTIS_GPU_NL_DUMP") && iter < 4) {
            // diagnostics: the first pass's rate matrices of the first active cell (tools/nl_dump_cmp.py)
            HIPCHK(hipStreamSynchronize(G.stream));
            std::vector<double> hA, hb, hn, hp, hpops, hcorr;
            std::vector<int32_t> hs;
            if (d2h_vec(hA, M.A, (size_t)cell2) || d2h_vec(hb, M.b, (size_t)cell1) || d2h_vec(hn, M.norm, (size_t)cell1) ||
                d2h_vec(hp, M.pv, (size_t)cell1) || d2h_vec(hs, M.status, (size_t)ne) || d2h_vec(hpops, d_pops, (size_t)nl) ||
                d2h_vec(hcorr, d_corr, (size_t)ntg))
              return ARTIS_ERR_HIP;
            const std::string path = std::string(getenv("ARTIS_GPU_NL_DUMP")) + "_p" + std::to_string(iter) + "_gpu.bin";
            if (FILE *fp = fopen(path.c_str(), "wb")) {
              const int32_t hdr[5] = {ne, cell1, (int32_t)cell2, nl, (int32_t)ntg};
              fwrite(hdr, sizeof hdr, 1, fp);
              fwrite(el_D.data(), 4, ne, fp);
              fwrite(hs.data(), 4, ne, fp);
              fwrite(hA.data(), 8, hA.size(), fp);
              fwrite(hb.data(), 8, hb.size(), fp);
              fwrite(hn.data(), 8, hn.size(), fp);
              fwrite(hp.data(), 8, hp.size(), fp);
              fwrite(hpops.data(), 8, hpops.size(), fp);
              fwrite(hcorr.data(), 8, hcorr.size(), fp);
              fclose(fp);
            }
          }
        }
        k_nl_store<<<(nch + 63) / 64, 64, 0, G.stream>>>(dK, dD, N, M, d_act, a0, nch);
        NLSTEP("k_nl_store");
      }
      if (int e2 = read_fail("solve_nlte_pops_element")) return e2;
      std::vector<int32_t> done;
      if (d2h_vec(done, M.done, nact)) return ARTIS_ERR_HIP;
      std::vector<int32_t> act2, actk2;
      for (int a = 0; a < nact; a++) {
        h_iters[k_of_mgi[act[a]]] = iter + 1;
        if (!done[a]) {
          act2.push_back(act[a]);
          actk2.push_back(actk[a]);
        }
      }
      act.swap(act2);
      actk.swap(actk2);
    }
  }
  // nt_ionization_ratecoeff of every listed cell, the cooling rates of the iterated ones
  if (R.nt_on) {
    k_nl_ntrates<<<(c->ncells + TB - 1) / TB, TB, 0, G.stream>>>(KN, N, S, N.mgi, c->ncells);
    HIPCHK(hipGetLastError());
  }
  NLSTEP("k_nl_ntrates (final)");
  if (int e2 = te_launch(d_nl, nnl, 2, nullptr)) return e2;
  NLSTEP("k_te_solve (cooling)");
#undef NLSTEP
  HIPCHK(hipEventRecord(G.ev1, G.stream));
  HIPCHK(hipEventSynchronize(G.ev1));
  {
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, G.ev2, G.ev1));
    G.last_nlte_ms = ms;
  }
  if (int e2 = read_fail("update_grid_nlte")) return e2;
  // success: every array back to the caller
  HIPCHK(hipMemcpy(c->TR, N.TR, npf * sizeof(float), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(c->W, N.W, npf * sizeof(float), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(c->TJ, N.TJ, npf * sizeof(float), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(c->Te, N.Te, npf * sizeof(float), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(c->nne, N.nne, npf * sizeof(float), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(c->nnetot, N.nnetot, npf * sizeof(float), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(c->groundlevelpop, N.gp, npi * sizeof(float), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(c->partfunct, N.pf, npi * sizeof(float), hipMemcpyDeviceToHost));
  if (ntl > 0) HIPCHK(hipMemcpy(c->nlte_pops, N.nlte, (size_t)np * ntl * sizeof(double), hipMemcpyDeviceToHost));
  if (nbins > 0) {
    HIPCHK(hipMemcpy(c->bin_TR, N.binTR, (size_t)np * nbins * sizeof(float), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(c->bin_W, N.binW, (size_t)np * nbins * sizeof(float), hipMemcpyDeviceToHost));
  }
  if (R.detailed_bf && nbf > 0)
    HIPCHK(hipMemcpy(c->bfrate_estimator, N.bfrate, (size_t)np * nbf * sizeof(float), hipMemcpyDeviceToHost));
  if (R.nt_on) {
    HIPCHK(hipMemcpy(c->nt_frac_heating, N.nt_fh, npf * sizeof(float), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(c->nt_frac_ionization, N.nt_fi, npf * sizeof(float), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(c->nt_frac_excitation, N.nt_fe, npf * sizeof(float), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(c->nt_nneperion_when_solved, N.nt_nneper, npf * sizeof(float), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(c->nt_timestep_last_solved, N.nt_tls, npf * sizeof(int32_t), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(c->nt_eff_ionpot, N.nt_effion, npi * sizeof(float), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(c->nt_fracdep_ionization_ion, N.nt_fracdep, npi * sizeof(double), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(c->nt_prob_num_auger, N.nt_prob, npi * A1 * sizeof(float), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(c->nt_ionenfrac_num_auger, N.nt_ionen, npi * A1 * sizeof(float), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(c->nt_ionization_ratecoeff, N.ntY, npi * sizeof(double), hipMemcpyDeviceToHost));
  }
  HIPCHK(hipMemcpy(c->totalcooling, d_totcool, npf * sizeof(double), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(c->cooling_contrib_ion, d_ccion, npi * sizeof(double), hipMemcpyDeviceToHost));
  if (c->heatingcoolingrates)
    HIPCHK(hipMemcpy(c->heatingcoolingrates, d_rates, npf * ARTIS_TE_NRATES * sizeof(double), hipMemcpyDeviceToHost));
  if (c->nlte_iterations)
    for (int k = 0; k < c->ncells; k++) c->nlte_iterations[c->mgi[k]] = h_iters[k];
  return 0;
}
double artis_gpu_last_nlte_ms(void) { return G.last_nlte_ms; }

int artis_gpu_abi_version(void) { return ARTIS_GPU_ABI_VERSION; }
const char *artis_gpu_last_error(void) { return G.last_error.c_str(); }
double artis_gpu_last_transport_ms(void) { return G.last_transport_ms; }
double artis_gpu_last_precompute_ms(void) { return G.last_precompute_ms; }
int64_t artis_gpu_last_rounds(void) { return G.last_rounds; }

// init_spectra (spectrum.cc:495-500): lower_freq and delta_freq are float arrays (spectrum.h:18-19), so the
// bin width every deltaE divides by is the float difference of the float lower edge
static inline double spec_delta_freq(double nu_min, double dlognu, int nnu) {
  const float lower_freq = (float)exp(log(nu_min) + (nnu * (dlognu)));
  return (float)(exp(log(nu_min) + ((nnu + 1) * (dlognu))) - lower_freq);
}
int artis_gpu_spectrum(int nnubins, int nprocs, double *spec_flux, double *lc_lum, double *lc_lumcmf) {
  if (!G.initialised) return ARTIS_ERR_NOT_INITIALISED;
  if (nnubins <= 0 || nprocs <= 0 || !spec_flux || !lc_lum || !lc_lumcmf) return ARTIS_ERR_BAD_ARGUMENT;
  const int nt = G.ntstep;
  // spectrum.cc:491-500 init_spectra: bin edges with the reference's expressions (host libm)
  const double nu_min = G.K.G.nu_min_r, nu_max = G.K.G.nu_max_r;
  const double dlognu = (log(nu_max) - log(nu_min)) / nnubins;
  std::vector<double> delta(nnubins);
  for (int nnu = 0; nnu < nnubins; nnu++)
    delta[nnu] = spec_delta_freq(nu_min, dlognu, nnu);
  const size_t nspec = (size_t)nt * nnubins;
  double *d = nullptr;
  HIPCHK(dmalloc((void **)&d, (nspec + 2 * (size_t)nt + nnubins) * sizeof(double)));
  double *d_spec = d, *d_lc = d + nspec, *d_lccmf = d_lc + nt, *d_delta = d_lccmf + nt;
  // every step below may fail; the scratch is released on all paths
  auto run = [&]() -> int {
    if (int rc = sync_ctx()) return rc;
    HIPCHK(hipMemsetAsync(d, 0, (nspec + 2 * (size_t)nt) * sizeof(double), G.stream));
    HIPCHK(hipMemcpyAsync(d_delta, delta.data(), nnubins * sizeof(double), hipMemcpyHostToDevice, G.stream));
    if (G.npkts > 0)
      k_spectrum<<<(unsigned)((G.npkts + 255) / 256), 256, 0, G.stream>>>(
          G.d_ctx, G.d_soa, G.npkts, nt, nnubins, dlognu, d_delta, (double)nprocs, d_spec, d_lc, d_lccmf);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(spec_flux, d_spec, nspec * sizeof(double), hipMemcpyDeviceToHost, G.stream));
    HIPCHK(hipMemcpyAsync(lc_lum, d_lc, nt * sizeof(double), hipMemcpyDeviceToHost, G.stream));
    HIPCHK(hipMemcpyAsync(lc_lumcmf, d_lccmf, nt * sizeof(double), hipMemcpyDeviceToHost, G.stream));
    HIPCHK(hipStreamSynchronize(G.stream));
    return 0;
  };
  const int rc = run();
  (void)hipStreamSynchronize(G.stream);
  (void)hipFree(d);
  return rc;
}
int artis_gpu_spectra(const artis_spectra_request *req, artis_spectra_out *out) {
  if (!G.initialised) return ARTIS_ERR_NOT_INITIALISED;
  if (!req || !out || req->nnubins <= 0 || req->nprocs <= 0 || req->abin < -1 || req->abin >= ARTIS_MABINS ||
      (!out->emission != !out->absorption) || (out->trueemission && !out->emission) ||
      ((out->stokes_emission || out->stokes_absorption) && !out->emission)) {
    G.last_error = "spectra: bad request (nnubins, nprocs, abin) or inconsistent emission/absorption arrays";
    return ARTIS_ERR_BAD_ARGUMENT;
  }
  const int nt = G.ntstep, nnb = req->nnubins;
  const int ioncount = G.nelements * G.maxnions, proccount = 2 * ioncount + 1;
  const double nu_min = G.K.G.nu_min_r, nu_max = G.K.G.nu_max_r;
  const double dlognu = (log(nu_max) - log(nu_min)) / nnb;  // spectrum.cc:352, 491-500 (host libm)
  std::vector<double> delta(nnb);
  for (int nnu = 0; nnu < nnb; nnu++)
    delta[nnu] = spec_delta_freq(nu_min, dlognu, nnu);
  const size_t nb = (size_t)nt * nnb;
  // device accumulators, in the order of the sections below
  struct Sec {
    double *host;
    size_t n;
  } secs[] = {{out->flux, nb},
              {out->emission, nb * proccount},
              {out->trueemission, nb * proccount},
              {out->absorption, nb * ioncount},
              {out->stokes_flux, 3 * nb},
              {out->stokes_emission, 3 * nb * proccount},
              {out->stokes_absorption, 3 * nb * ioncount},
              {out->lc_lum, (size_t)nt},
              {out->lc_lumcmf, (size_t)nt},
              {out->gamma_lc_lum, (size_t)nt},
              {out->gamma_lc_lumcmf, (size_t)nt}};
  constexpr int NSEC = sizeof(secs) / sizeof(secs[0]);
  size_t total = nnb;  // delta_freq first
  for (const Sec &x : secs)
    if (x.host) total += x.n;
  double *d = nullptr;
  HIPCHK(dmalloc((void **)&d, total * sizeof(double)));
  double *dptr[NSEC];
  size_t off = nnb;
  for (int k = 0; k < NSEC; k++) {
    dptr[k] = secs[k].host ? d + off : nullptr;
    if (secs[k].host) off += secs[k].n;
  }
  auto run = [&]() -> int {
    if (int rc = sync_ctx()) return rc;
    HIPCHK(hipMemsetAsync(d + nnb, 0, (total - nnb) * sizeof(double), G.stream));
    HIPCHK(hipMemcpyAsync(d, delta.data(), nnb * sizeof(double), hipMemcpyHostToDevice, G.stream));
    SpecArgs A{};
    A.nnubins = nnb;
    A.nprocs = req->nprocs;
    A.abin = req->abin;
    A.ntstep = nt;
    A.proccount = proccount;
    A.ioncount = ioncount;
    A.maxnions = G.maxnions;
    A.nbf = G.K.T.nbf;
    for (int k = 0; k < 3; k++) A.syn_dir[k] = req->syn_dir[k];
    A.dlognu = dlognu;
    A.delta_freq = d;
    A.bf_col = G.d_bfcol;
    A.line_elem = G.K.T.line_elem;
    A.line_ion = G.K.T.line_ion;
    A.flux = dptr[0];
    A.emission = dptr[1];
    A.trueemission = dptr[2];
    A.absorption = dptr[3];
    A.sflux = dptr[4];
    A.semission = dptr[5];
    A.sabsorption = dptr[6];
    A.lc = dptr[7];
    A.lccmf = dptr[8];
    A.glc = dptr[9];
    A.glccmf = dptr[10];
    if (G.npkts > 0)
      k_spectra<<<(unsigned)((G.npkts + 255) / 256), 256, 0, G.stream>>>(G.d_ctx, G.d_soa, G.npkts, A);
    HIPCHK(hipGetLastError());
    std::vector<double> h;
    for (int k = 0; k < NSEC; k++) {
      if (!secs[k].host) continue;
      h.resize(secs[k].n);
      HIPCHK(hipMemcpyAsync(h.data(), dptr[k], secs[k].n * sizeof(double), hipMemcpyDeviceToHost, G.stream));
      HIPCHK(hipStreamSynchronize(G.stream));
      for (size_t j = 0; j < secs[k].n; j++) secs[k].host[j] += h[j];
    }
    return 0;
  };
  const int rc = run();
  (void)hipStreamSynchronize(G.stream);
  (void)hipFree(d);
  return rc;
}

int artis_gpu_vpkt_init(const artis_vpkt_params *vp) {
  if (!G.initialised) return ARTIS_ERR_NOT_INITIALISED;
  if (!vp || vp->nobs <= 0 || vp->nspectra <= 0 || vp->nspectra > ARTIS_VPKT_MAX_SPECTRA || vp->nrange < 0 ||
      vp->nrange > ARTIS_VPKT_MRANGE || vp->vmtbins <= 0 || vp->vmnubins <= 0 || !vp->nz_obs || !vp->phi_obs ||
      !vp->exclude || vp->nprocs <= 0 || vp->spawn_capacity < 0 ||
      (vp->vgrid_flag == 1 && (vp->nrange_grid < 0 || vp->nrange_grid > ARTIS_VPKT_MRANGE_GRID ||
                               vp->ny_vgrid <= 0 || vp->nz_vgrid <= 0))) {
    G.last_error = "vpkt_init: bad virtual-packet parameters";
    return ARTIS_ERR_BAD_ARGUMENT;
  }
  static_assert(VPKT_MAX_SPECTRA == ARTIS_VPKT_MAX_SPECTRA && VPKT_MRANGE == ARTIS_VPKT_MRANGE &&
                    VPKT_MRANGE_GRID == ARTIS_VPKT_MRANGE_GRID,
                "device and ABI vpkt limits differ");
  DevVpkt V{};
  V.nobs = vp->nobs;
  V.nspectra = vp->nspectra;
  V.vmtbins = vp->vmtbins;
  V.vmnubins = vp->vmnubins;
  V.nrange = vp->nrange;
  V.vgrid_flag = vp->vgrid_flag;
  V.nrange_grid = vp->vgrid_flag == 1 ? vp->nrange_grid : 0;
  V.ny_vgrid = vp->ny_vgrid;
  V.nz_vgrid = vp->nz_vgrid;
  V.nprocs = vp->nprocs;
  for (int i = 0; i < VPKT_MAX_SPECTRA; i++) V.exclude[i] = i < vp->nspectra ? vp->exclude[i] : 0.;
  V.tmin_vspec = vp->tmin_vspec;
  V.tmax_vspec = vp->tmax_vspec;
  V.numin_vspec = vp->numin_vspec;
  V.numax_vspec = vp->numax_vspec;
  V.tmin_input = vp->tmin_vspec_input;
  V.tmax_input = vp->tmax_vspec_input;
  for (int i = 0; i < VPKT_MRANGE; i++) {
    V.numin_input[i] = vp->numin_vspec_input[i];
    V.numax_input[i] = vp->numax_vspec_input[i];
  }
  V.tau_max = vp->tau_max_vpkt;
  V.tmin_grid = vp->tmin_grid;
  V.tmax_grid = vp->tmax_grid;
  for (int i = 0; i < VPKT_MRANGE_GRID; i++) {
    V.nu_grid_min[i] = vp->nu_grid_min[i];
    V.nu_grid_max[i] = vp->nu_grid_max[i];
  }
  // observer vectors (vpkt.cc:863-865) and the float bin edges of init_vspecpol (vpkt.cc:425-436), host libm
  std::vector<double> obs(3 * (size_t)vp->nobs);
  for (int b = 0; b < vp->nobs; b++) {
    const double nz = vp->nz_obs[b], phi = vp->phi_obs[b];
    obs[3 * b] = sqrt(1 - nz * nz) * cos(phi);
    obs[3 * b + 1] = sqrt(1 - nz * nz) * sin(phi);
    obs[3 * b + 2] = nz;
  }
  V.dlogt = (log(vp->tmax_vspec) - log(vp->tmin_vspec)) / vp->vmtbins;
  V.dlognu = (log(vp->numax_vspec) - log(vp->numin_vspec)) / vp->vmnubins;
  std::vector<float> delta_t(vp->vmtbins), delta_freq(vp->vmnubins);
  for (int n = 0; n < vp->vmtbins; n++) {
    const float lower = (float)exp(log(vp->tmin_vspec) + (n * (V.dlogt)));
    delta_t[n] = (float)(exp(log(vp->tmin_vspec) + ((n + 1) * (V.dlogt))) - lower);
  }
  for (int m = 0; m < vp->vmnubins; m++) {
    const float lower = (float)exp(log(vp->numin_vspec) + (m * (V.dlognu)));
    delta_freq[m] = (float)(exp(log(vp->numin_vspec) + ((m + 1) * (V.dlognu))) - lower);
  }
  const std::vector<int32_t> &anum = G.h_anumber;
  int rc = 0;
  rc |= dupload(&V.obs, obs.data(), obs.size());
  rc |= dupload(&V.delta_t, delta_t.data(), delta_t.size());
  rc |= dupload(&V.delta_freq, delta_freq.data(), delta_freq.size());
  rc |= dupload(&V.anumber, anum.data(), anum.size());
  {
    // per line, the spectra whose optical depth its opacity enters (vpkt.cc:283-294: exclude -1 drops every
    // line, exclude Z the lines of element Z); padded for the walk's 16-line windows
    const size_t nli = G.h_line_elem.size();
    std::vector<uint8_t> mask((nli + 15) / 16 * 16 + 16, 0);
    for (size_t li = 0; li < nli; li++) {
      const int an = anum.empty() ? 0 : anum[G.h_line_elem[li]];
      uint8_t m = 0;
      for (int ind = 0; ind < vp->nspectra; ind++)
        if (V.exclude[ind] != -1 && (an != V.exclude[ind])) m |= (uint8_t)(1u << ind);
      mask[li] = m;
    }
    rc |= dupload(&V.line_mask, mask.data(), mask.size());
  }
  V.vstokes_stride = (int64_t)vp->vmtbins * vp->nobs * vp->nspectra * vp->vmnubins;
  V.vgrid_stride = (vp->vgrid_flag == 1) ? (int64_t)vp->ny_vgrid * vp->nz_vgrid * vp->nrange_grid * vp->nobs : 0;
  rc |= dalloc(&V.vstokes, (size_t)(3 * V.vstokes_stride));
  rc |= dalloc(&V.vgrid, (size_t)std::max<int64_t>(3 * V.vgrid_stride, 1));
  rc |= dalloc(&V.ctr, 8);
  rc |= dalloc(&V.spawn_ctr, 2);
  V.ovf_cap = (uint32_t)((int64_t)G.wave_grid * WAVE_BLOCK);
  rc |= dalloc(&V.ovf, (size_t)V.ovf_cap * VPKT_SPAWN_WORDS);
  rc |= dalloc(&V.ovf_ctr, 1);
  rc |= dalloc(&V.full, 1);
  if (!G.d_qsnap) rc |= dalloc(&G.d_qsnap, 1);
  if (!G.h_vfull) HIPCHK(hipHostMalloc((void **)&G.h_vfull, sizeof(uint32_t), hipHostMallocDefault));
  if (rc) return ARTIS_ERR_HIP;
  V.spawn = G.d_vpkt_spawn;
  V.cap = G.vpkt_spawn_cap;
  V.on = 1;
  // the negative-coefficient flag belongs to the per-cell tables (read back by artis_gpu_upload_cellstate), not to
  // the vpkt parameters: keep it when vpkt_init runs after an upload
  V.neg_coef = G.K.V.neg_coef;
  G.K.V = V;
  G.vpkt_cap_param = vp->spawn_capacity;
  return artis_gpu_vpkt_zero();
}

int artis_gpu_vpkt_zero(void) {
  if (!G.initialised) return ARTIS_ERR_NOT_INITIALISED;
  const DevVpkt &V = G.K.V;
  if (!V.on) return ARTIS_ERR_BAD_ARGUMENT;
  HIPCHK(hipMemsetAsync(V.vstokes, 0, (size_t)3 * V.vstokes_stride * sizeof(double), G.stream));
  if (V.vgrid_stride) HIPCHK(hipMemsetAsync(V.vgrid, 0, (size_t)3 * V.vgrid_stride * sizeof(double), G.stream));
  HIPCHK(hipMemsetAsync(V.ctr, 0, 8 * sizeof(unsigned long long), G.stream));
  HIPCHK(hipMemsetAsync(V.spawn_ctr, 0, 2 * sizeof(uint32_t), G.stream));
  HIPCHK(hipStreamSynchronize(G.stream));
  return 0;
}

int artis_gpu_vpkt_download(artis_vpkt_result *out, int reset_counters) {
  if (!G.initialised) return ARTIS_ERR_NOT_INITIALISED;
  const DevVpkt &V = G.K.V;
  if (!V.on || !out || !out->vstokes_i || !out->vstokes_q || !out->vstokes_u) return ARTIS_ERR_BAD_ARGUMENT;
  if (V.vgrid_stride && (!out->vgrid_i || !out->vgrid_q || !out->vgrid_u)) return ARTIS_ERR_BAD_ARGUMENT;
  HIPCHK(hipStreamSynchronize(G.stream));
  std::vector<double> h((size_t)3 * std::max(V.vstokes_stride, V.vgrid_stride));
  HIPCHK(hipMemcpy(h.data(), V.vstokes, (size_t)3 * V.vstokes_stride * sizeof(double), hipMemcpyDeviceToHost));
  double *dst[3] = {out->vstokes_i, out->vstokes_q, out->vstokes_u};
  for (int c = 0; c < 3; c++)
    for (int64_t j = 0; j < V.vstokes_stride; j++) dst[c][j] += h[c * V.vstokes_stride + j];
  if (V.vgrid_stride) {
    HIPCHK(hipMemcpy(h.data(), V.vgrid, (size_t)3 * V.vgrid_stride * sizeof(double), hipMemcpyDeviceToHost));
    double *gd[3] = {out->vgrid_i, out->vgrid_q, out->vgrid_u};
    for (int c = 0; c < 3; c++)
      for (int64_t j = 0; j < V.vgrid_stride; j++) gd[c][j] += h[c * V.vgrid_stride + j];
  }
  unsigned long long ctr[8];
  HIPCHK(hipMemcpy(ctr, V.ctr, sizeof(ctr), hipMemcpyDeviceToHost));
  out->nvpkt += (int64_t)ctr[0];
  out->nvpkt_esc1 += (int64_t)ctr[1];
  out->nvpkt_esc2 += (int64_t)ctr[2];
  out->nvpkt_esc3 += (int64_t)ctr[3];
  if (reset_counters) HIPCHK(hipMemset(V.ctr, 0, 4 * sizeof(unsigned long long)));
  return 0;
}

int artis_gpu_vpkt_last_stats(double *ms, int64_t *spawns, int64_t *traces) {
  if (ms) *ms = G.last_vpkt_ms;
  if (spawns) *spawns = G.last_vpkt_spawns;
  if (traces) *traces = G.last_vpkt_traces;
  return 0;
}

int64_t artis_gpu_vpkt_last_drains(void) { return G.vpkt_drains; }

int artis_gpu_vpkt_last_work(int64_t work[4]) {
  if (!work) return ARTIS_ERR_BAD_ARGUMENT;
  for (int i = 0; i < 4; i++) work[i] = G.last_vpkt_work[i];
  return 0;
}

int artis_gpu_last_kernel_times(double ms[4], int64_t launches[4]) {
  for (int c = 0; c < 4; c++) {
    ms[c] = G.last_kernel_ms[c];
    launches[c] = G.last_kernel_launches[c];
  }
  for (int c = 4; c < ARTIS_KCLASS_COUNT; c++) {  // (classes 4-6 are class 3's parts)
    ms[3] += G.last_kernel_ms[c];
    launches[3] += G.last_kernel_launches[c];
  }
  return 0;
}
int artis_gpu_last_kernel_class_times(double ms[ARTIS_KCLASS_COUNT], int64_t launches[ARTIS_KCLASS_COUNT]) {
  if (!ms || !launches) return ARTIS_ERR_BAD_ARGUMENT;
  for (int c = 0; c < ARTIS_KCLASS_COUNT; c++) {
    ms[c] = G.last_kernel_ms[c];
    launches[c] = G.last_kernel_launches[c];
  }
  return 0;
}
int artis_gpu_table_info(int64_t out[ARTIS_TABLE_INFO_COUNT]) {
  if (!G.initialised) return ARTIS_ERR_NOT_INITIALISED;
  const DevCells &C = G.K.C;
  out[0] = C.n_nonempty;
  out[1] = C.linecoef_rows;
  out[2] = (int64_t)C.linecoef_rows * C.linecoef_stride * 8;
  out[3] = C.ma_rows;
  out[4] = (int64_t)C.ma_rows * C.ma_key_stride * 2;
  out[5] = C.marates ? (int64_t)C.n_nonempty * G.K.T.nlevels_total * ARTIS_MA_ACTION_COUNT * 8 : 0;
  out[6] = G.ma_acts_cached;
  out[7] = G.ma_acts_total;
  out[8] = C.ma_level_mode ? G.ma_level_records : 0;
  out[9] = C.ma_level_mode ? G.ma_level_lines * 128 : 0;
  out[10] = C.ma_level_mode ? (int64_t)G.ma_pool_lines * 128 : 0;
  return 0;
}

int artis_gpu_last_work_counts(int64_t out[ARTIS_WORK_COUNT]) {
  for (int k = 0; k < ARTIS_WORK_COUNT; k++) out[k] = G.last_work[k];
  return 0;
}

void artis_gpu_finalize(void) {
  if (!G.initialised) return;
  artis_gpu_comm_finalize();
  dfree(G.d_redblock);
  for (void *p : G.allocs) (void)hipFree(p);
  G.allocs.clear();
  free_packets();
  if (G.h_ctr) (void)hipHostFree(G.h_ctr);
  if (G.h_vfull) (void)hipHostFree(G.h_vfull);
  if (G.d_vpkt_spawn) (void)hipFree(G.d_vpkt_spawn);
  for (uint32_t *a : {G.d_vkey, G.d_vkey2, G.d_vidx, G.d_vperm})
    if (a) (void)hipFree(a);
  if (G.d_vsort_tmp) (void)hipFree(G.d_vsort_tmp);
  if (G.h_vcount) (void)hipHostFree(G.h_vcount);
  for (hipEvent_t e : G.vev) (void)hipEventDestroy(e);
  for (hipEvent_t e : G.tev) (void)hipEventDestroy(e);
  for (int r = 0; r < 2; r++)
    if (G.ev_round[r]) (void)hipEventDestroy(G.ev_round[r]);
  if (G.ev0) (void)hipEventDestroy(G.ev0);
  if (G.ev1) (void)hipEventDestroy(G.ev1);
  if (G.ev2) (void)hipEventDestroy(G.ev2);
  if (G.stream) (void)hipStreamDestroy(G.stream);
  G = Engine();
}

// Option values the engine does not propagate are refused at init instead of being accepted and ignored: the
// reference's own input checks (input.cc:1976-1982 do_rlc_est in 0..3, grid.cc:627-677 opacity_case 0..5) plus
// every switch being 0 / 1.  Runs before any HIP call.
static const char *unsupported_run_param(const artis_run_params *rp) {
  auto flag = [](int32_t v) { return v == 0 || v == 1; };
  if (rp->do_rlc_est < 0 || rp->do_rlc_est > 3) return "do_rlc_est must be 0..3 (input.txt line 9 is 0..4)";
  if (rp->opacity_case < 0 || rp->opacity_case > 5) return "opacity_case must be 0..5";
  if (!flag(rp->do_r_lc) || !flag(rp->pol_dipole) || !flag(rp->relativistic_doppler) || !flag(rp->record_linestat) ||
      !flag(rp->instant_particle_deposition) || !flag(rp->nt_solve_spencerfano) || !flag(rp->nlte_pops_on) ||
      !flag(rp->multibin_radfield) || !flag(rp->detailed_bf_estimators) || !flag(rp->no_lut_photoion) ||
      !flag(rp->no_lut_bfheating) || !flag(rp->nt_on) || !flag(rp->comp_est))
    return "a boolean run parameter (do_r_lc, pol_dipole, relativistic_doppler, record_linestat, "
           "instant_particle_deposition, nt_solve_spencerfano, nlte_pops_on, multibin_radfield, "
           "detailed_bf_estimators, no_lut_photoion, no_lut_bfheating, nt_on, comp_est) is not 0 or 1";
  if (rp->n_kpktdiffusion_timesteps < 0 || !(rp->kpktdiffusion_timescale >= 0.f))
    return "kpkt diffusion parameters must be >= 0";
  if (!(rp->max_path_step > 0.)) return "max_path_step must be > 0";
  if (!std::isfinite(rp->gamma_grey) || !(rp->minpop >= 0.) || rp->rank < 0)
    return "gamma_grey must be finite, minpop >= 0, rank >= 0";
  return nullptr;
}

int artis_gpu_init(int device, const artis_atomic_tables *a, const artis_geometry *g, const artis_run_params *rp) {
  if (!a || !g || !rp) return ARTIS_ERR_BAD_ARGUMENT;
  if (const char *why = unsupported_run_param(rp)) {
    G.last_error = why;
    return ARTIS_ERR_UNSUPPORTED;
  }
  if (G.initialised) artis_gpu_finalize();
  if (g->grid_type != ARTIS_GRID_UNIFORM && g->grid_type != ARTIS_GRID_SPHERICAL1D) {
    G.last_error = "grid_type must be GRID_UNIFORM or GRID_SPHERICAL1D";
    return ARTIS_ERR_UNSUPPORTED;
  }
  if (g->grid_type == ARTIS_GRID_SPHERICAL1D) {
    // spherical1d_grid_setup (grid.cc:2104-2131): one propagation cell per model shell, cellindex == mgi (or
    // npts_model for an empty shell), the radial extent at tmin of every shell given
    bool ok = g->ncoordgrid[0] == g->ngrid && g->ncoordgrid[1] == 1 && g->ncoordgrid[2] == 1 &&
              g->ngrid == g->npts_model && g->modelcell_wid_init && g->cell_mgi && g->cell_pos_min;
    for (int c = 0; ok && c < g->ngrid; c++)
      ok = (g->cell_mgi[c] == c || g->cell_mgi[c] == g->npts_model) && g->modelcell_wid_init[c] > 0 &&
           g->cell_pos_min[3 * (int64_t)c] >= 0;
    if (!ok) {
      G.last_error = "GRID_SPHERICAL1D needs ncoordgrid = {npts_model, 1, 1}, cell_mgi[c] in {c, npts_model}, "
                     "modelcell_wid_init > 0 and radii >= 0";
      return ARTIS_ERR_BAD_ARGUMENT;
    }
  }
  G.device = device;
  HIPCHK(hipSetDevice(device));
  HIPCHK(hipStreamCreateWithFlags(&G.stream, hipStreamNonBlocking));
  HIPCHK(hipEventCreate(&G.ev0));
  HIPCHK(hipEventCreate(&G.ev1));
  HIPCHK(hipEventCreate(&G.ev2));
  for (int r = 0; r < 2; r++) HIPCHK(hipEventCreateWithFlags(&G.ev_round[r], hipEventDisableTiming));
  HIPCHK(hipHostMalloc((void **)&G.h_ctr, 2 * NQUEUES * 2 * sizeof(uint32_t), hipHostMallocDefault));
  {
    int ncu = 256;
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device);
    G.wave_grid = ncu * 8;  // 32 waves per CU of 256-thread blocks; late blocks find the queue drained
    // (tests: ARTIS_GPU_WAVE_GRID=<blocks>, a multiple of 8, shrinks the persistent grids and the vpkt overflow records)
    if (const char *wg = getenv("ARTIS_GPU_WAVE_GRID")) G.wave_grid = std::max(8, atoi(wg) / 8 * 8);
    const char *eng = getenv("ARTIS_GPU_ENGINE");
    G.use_megakernel = eng && std::string(eng) == "mega";
    // cell binning of the macro-atom queue (measured 5-15 % faster walks: lanes of a wave share a cell's
    // records) is on; per-XCD queue ranges measured neutral-to-negative and are off unless asked for
    const char *b = getenv("ARTIS_GPU_MA_BIN");
    G.W.ma_binned = !(b && b[0] == '0');
    // cell binning of the R queue before k_rpkt: measured no faster k_rpkt (1114 vs 1106 ms per bench step) and
    // ~250 ms more binning per step (profiles/r03g_ab.txt), so off unless asked for (ARTIS_GPU_R_BIN=1)
    const char *rb = getenv("ARTIS_GPU_R_BIN");
    G.r_binned = rb && rb[0] == '1';
    const char *rw = getenv("ARTIS_GPU_RPKT_WALK");
    G.rpkt_walk = rw ? (rw[0] == '1' ? 1 : 0) : -1;
    const char *rc_ = getenv("ARTIS_GPU_RPKT_COOP");
    G.rpkt_coop = !(rc_ && rc_[0] == '0');
    const char *mp = getenv("ARTIS_GPU_MA_PRE");
    G.ma_pre_on = !(mp && mp[0] == '0');
    const char *mf = getenv("ARTIS_GPU_MF_REC");
    G.mf_rec_on = !(mf && mf[0] == '0');
    const char *bp = getenv("ARTIS_GPU_BIN_PUSH");
    G.bin_push_on = !(bp && bp[0] == '0');
    const char *bb = getenv("ARTIS_GPU_MA_BIN_BLK");
    G.ma_bin_blk = !(bb && bb[0] == '0');
    const char *xr = getenv("ARTIS_GPU_MA_XCD");
    G.W.ma_ranges = (xr && xr[0] == '1') ? 8 : 1;
    const char *rf = getenv("ARTIS_GPU_REFILL");
    G.W.refill_min = rf ? std::max(1, std::min(64, atoi(rf))) : 32;
    // k_ma refills from one coalesced ticket read, so it refills early (1e7-packet bench, before tickets:
    // 32 idle lanes 2212 ms, 16: 2064 ms, 8: 2042 ms; round 5, with the line-0 suffix and the F-queue records:
    // 4: 2578 ms, 8: 1694, 12: 1559, 14: 1568, 16: 1581, 20: 1617, 24: 1659; profiles/r5s_refill_sweep.txt)
    const char *rfm = getenv("ARTIS_GPU_REFILL_MA");
    G.W.refill_ma = rfm ? std::max(1, std::min(64, atoi(rfm))) : 12;
    const char *oc = getenv("ARTIS_GPU_MA_OCC");
    G.ma_occ = (oc && oc[0] == '8') ? 8 : 1;
    const char *cm = getenv("ARTIS_GPU_MA_COOP_MAX");
    G.W.coop_max = cm ? std::max(1, std::min(64, atoi(cm))) : 64;
    // level mode: the jumps without a record made inline by k_ma's wave (ARTIS_GPU_MA_LEVEL_COOP=1), or parked
    // for k_ma_exact (default: k_ma keeps the row kernel's register budget)
    const char *lc = getenv("ARTIS_GPU_MA_LEVEL_COOP");
    G.ma_level_coop = lc && lc[0] == '1';
  }
  G.params = *rp;
  G.h_anumber.assign(a->nelements, 0);
  if (a->elem_anumber) G.h_anumber.assign(a->elem_anumber, a->elem_anumber + a->nelements);
  G.h_ion_ionpot.assign(a->nions_total, 0.);
  if (a->ion_ionpot) G.h_ion_ionpot.assign(a->ion_ionpot, a->ion_ionpot + a->nions_total);
  DevTab &T = G.K.T;
  T.nelements = a->nelements;
  T.maxnions = a->maxnions;
  T.nions_total = a->nions_total;
  T.nlevels_total = a->nlevels_total;
  T.nlines = a->nlines;
  T.nbf = a->nbfcontinua;
  T.nbfg = a->nbfcontinua_ground;
  T.ncoolingterms = a->ncoolingterms;
  T.nphixspoints = a->nphixspoints;
  T.phixs_file_version = a->phixs_file_version;
  T.tablesize = a->tablesize;
  T.nphixsnuincrement = a->nphixsnuincrement;
  T.last_phixs_nuovernuedge = a->last_phixs_nuovernuedge;
  T.mintemp = a->mintemp;
  T.T_step_log = (log(a->maxtemp) - log(a->mintemp)) / (a->tablesize - 1.);  // ratecoeff.cc:1004
  const int ne = a->nelements, ni = a->nions_total, nl = a->nlevels_total, nli = a->nlines, nb = a->nbfcontinua;
  const int64_t nup = sum_i32(a->level_nuptrans, nl), ndown = sum_i32(a->level_ndowntrans, nl);
  const int64_t ntg = sum_i32(a->level_nphixstargets, nl);
  T.ntargets_total = (int)ntg;
  int64_t ntables = 0;
  for (int i = 0; i < nl; i++) ntables = std::max<int64_t>(ntables, a->level_phixstable[i] + 1);
  int rc = 0;
  rc |= dupload(&T.elem_nions, a->elem_nions, ne);
  rc |= dupload(&T.elem_uniqueionoffset, a->elem_uniqueionoffset, ne);
  rc |= dupload(&T.ion_ionstage, a->ion_ionstage, ni);
  rc |= dupload(&T.ion_nlevels, a->ion_nlevels, ni);
  rc |= dupload(&T.ion_uniqueleveloffset, a->ion_uniqueleveloffset, ni);
  rc |= dupload(&T.ion_ionisinglevels, a->ion_ionisinglevels, ni);
  rc |= dupload(&T.ion_maxrecombininglevel, a->ion_maxrecombininglevel, ni);
  rc |= dupload(&T.ion_coolingoffset, a->ion_coolingoffset, ni);
  rc |= dupload(&T.ion_ncoolingterms, a->ion_ncoolingterms, ni);
  std::vector<int32_t> ion_element(ni), level_ui(nl);
  for (int e = 0; e < ne; e++)
    for (int i = 0; i < a->elem_nions[e]; i++) ion_element[a->elem_uniqueionoffset[e] + i] = e;
  for (int ui = 0; ui < ni; ui++)
    for (int l = 0; l < a->ion_nlevels[ui]; l++) level_ui[a->ion_uniqueleveloffset[ui] + l] = ui;
  rc |= dupload(&T.ion_element, ion_element.data(), ni);
  rc |= dupload(&T.level_ui, level_ui.data(), nl);
  rc |= dupload(&T.level_epsilon, a->level_epsilon, nl);
  rc |= dupload(&T.level_stat_weight, a->level_stat_weight, nl);
  rc |= dupload(&T.level_nuptrans, a->level_nuptrans, nl);
  rc |= dupload(&T.level_uptrans_offset, a->level_uptrans_offset, nl);
  rc |= dupload(&T.level_ndowntrans, a->level_ndowntrans, nl);
  rc |= dupload(&T.level_downtrans_offset, a->level_downtrans_offset, nl);
  rc |= dupload(&T.level_nphixstargets, a->level_nphixstargets, nl);
  rc |= dupload(&T.level_phixstargets_offset, a->level_phixstargets_offset, nl);
  rc |= dupload(&T.level_cont_index, a->level_cont_index, nl);
  rc |= dupload(&T.level_closestgroundlevelcont, a->level_closestgroundlevelcont, nl);
  rc |= dupload(&T.level_phixstable, a->level_phixstable, nl);
  rc |= dupload(&T.uptrans_lineindex, a->uptrans_lineindex, nup);
  rc |= dupload(&T.downtrans_lineindex, a->downtrans_lineindex, ndown);
  rc |= dupload(&T.phixstarget_levelindex, a->phixstarget_levelindex, ntg);
  rc |= dupload(&T.phixstarget_probability, a->phixstarget_probability, ntg);
  rc |= dupload(&T.phixs_xs, a->phixs_xs, (size_t)ntables * a->nphixspoints);
  rc |= dupload(&T.line_nu, a->line_nu, nli);
  {
    std::vector<double> nu8((size_t)(nli + 15) / 16 * 16 + 16, 0.);  // (padded for 16-line windows, k_vpkt)
    std::copy(a->line_nu, a->line_nu + nli, nu8.begin());
    rc |= dupload(&T.line_nu8, nu8.data(), nu8.size());
  }
  rc |= dupload(&T.line_A, a->line_einstein_A, nli);
  rc |= dupload(&T.line_f, a->line_osc_strength, nli);
  rc |= dupload(&T.line_coll, a->line_coll_str, nli);
  rc |= dupload(&T.line_elem, a->line_elementindex, nli);
  G.h_line_elem.assign(a->line_elementindex, a->line_elementindex + nli);
  rc |= dupload(&T.line_ion, a->line_ionindex, nli);
  rc |= dupload(&T.line_upper, a->line_upperlevelindex, nli);
  rc |= dupload(&T.line_lower, a->line_lowerlevelindex, nli);
  rc |= dupload(&T.line_forbidden, a->line_forbidden, nli);
  // per-line Sobolev coefficients, evaluated on the host with the same expression as rpkt.cc:179-181
  std::vector<LineTau> lt(nli);
  for (int li = 0; li < nli; li++) {
    const int e = a->line_elementindex[li], i = a->line_ionindex[li];
    const int off = a->ion_uniqueleveloffset[a->elem_uniqueionoffset[e] + i];
    const int ulo = off + a->line_lowerlevelindex[li], uup = off + a->line_upperlevelindex[li];
    const double nu_trans = a->line_nu[li];
    const double A_ul = a->line_einstein_A[li];
    const double B_ul = ARTIS_CLIGHTSQUAREDOVERTWOH / pow(nu_trans, 3) * A_ul;
    const double B_lu = (double)a->level_stat_weight[uup] / (double)a->level_stat_weight[ulo] * B_ul;
    lt[li] = {nu_trans, B_ul, B_lu, ulo, uup};
  }
  rc |= dupload(&T.line_tau, lt.data(), nli);
  // macro-atom per-line constants (macroatom.cc:518-522, 563-566; radfield.h:47; macroatom.h:93,130)
  std::vector<LineMA> lm(nli);
  for (int li = 0; li < nli; li++) {
    const int ulo = lt[li].ul_lower, uup = lt[li].ul_upper;
    const double epsilon_trans = a->level_epsilon[uup] - a->level_epsilon[ulo];
    const double nu_trans = epsilon_trans / ARTIS_H;
    const double A_ul = a->line_einstein_A[li];
    const double B_ul = ARTIS_CLIGHTSQUAREDOVERTWOH / pow(nu_trans, 3) * A_ul;
    const double B_lu = (double)a->level_stat_weight[uup] / (double)a->level_stat_weight[ulo] * B_ul;
    lm[li] = {B_ul, B_lu, pow(nu_trans, 3), pow(ARTIS_H_IONPOT / epsilon_trans, 2)};
  }
  rc |= dupload(&T.line_ma, lm.data(), nli);
  {
    // packed collisional-excitation terms (TeExcItem) indexed like uptrans_lineindex
    size_t nitems = 0;
    for (int ul = 0; ul < nl; ul++)
      nitems = std::max(nitems, (size_t)a->level_uptrans_offset[ul] + (size_t)a->level_nuptrans[ul]);
    std::vector<TeExcItem> items(std::max<size_t>(nitems, 1));
    for (int ui = 0; ui < a->nions_total; ui++) {
      const int ul0 = a->ion_uniqueleveloffset[ui];
      for (int l = 0; l < a->ion_nlevels[ui]; l++) {
        const int ul = ul0 + l;
        for (int ii = 0; ii < a->level_nuptrans[ul]; ii++) {
          const int j = a->level_uptrans_offset[ul] + ii;
          const int li = a->uptrans_lineindex[j];
          const int uu = ul0 + a->line_upperlevelindex[li];
          TeExcItem &x = items[j];
          x.epsilon_trans = a->level_epsilon[uu] - a->level_epsilon[ul];
          x.P2 = lm[li].P2;
          x.coll_str = a->line_coll_str[li];
          x.osc_f = a->line_osc_strength[li];
          x.upper_sw = a->level_stat_weight[uu];
          x.forbidden = a->line_forbidden[li];
        }
      }
    }
    rc |= dupload(&T.exc_items, items.data(), items.size());
  }
  {
    // k_marates' packed transition items (MaDownItem / MaUpItem) indexed like downtrans_lineindex / uptrans_lineindex
    size_t nd_items = 1, nu_items = 1;
    for (int ul = 0; ul < nl; ul++) {
      nd_items = std::max(nd_items, (size_t)a->level_downtrans_offset[ul] + (size_t)a->level_ndowntrans[ul]);
      nu_items = std::max(nu_items, (size_t)a->level_uptrans_offset[ul] + (size_t)a->level_nuptrans[ul]);
    }
    std::vector<MaDownItem> di(nd_items);
    std::vector<MaUpItem> ui_(nu_items);
    for (int ui = 0; ui < a->nions_total; ui++) {
      const int ul0 = a->ion_uniqueleveloffset[ui];
      for (int l = 0; l < a->ion_nlevels[ui]; l++) {
        const int ul = ul0 + l;
        for (int j = 0; j < a->level_ndowntrans[ul]; j++) {
          const int li = a->downtrans_lineindex[a->level_downtrans_offset[ul] + j];
          const int lo = a->line_lowerlevelindex[li];
          MaDownItem &x = di[a->level_downtrans_offset[ul] + j];
          x = MaDownItem{};
          x.lower = lo;
          x.forbidden = a->line_forbidden[li];
          x.A = a->line_einstein_A[li];
          x.coll = a->line_coll_str[li];
          x.osc_f = a->line_osc_strength[li];
          x.lower_sw = a->level_stat_weight[ul0 + lo];
          x.eps_target = a->level_epsilon[ul0 + lo];
          x.B_ul = lm[li].B_ul;
          x.B_lu = lm[li].B_lu;
          x.P2 = lm[li].P2;
        }
        for (int j = 0; j < a->level_nuptrans[ul]; j++) {
          const int li = a->uptrans_lineindex[a->level_uptrans_offset[ul] + j];
          const int up = a->line_upperlevelindex[li];
          MaUpItem &x = ui_[a->level_uptrans_offset[ul] + j];
          x = MaUpItem{};
          x.upper = up;
          x.forbidden = a->line_forbidden[li];
          x.coll = a->line_coll_str[li];
          x.osc_f = a->line_osc_strength[li];
          x.upper_sw = a->level_stat_weight[ul0 + up];
          x.eps_upper = a->level_epsilon[ul0 + up];
          x.B_ul = lm[li].B_ul;
          x.B_lu = lm[li].B_lu;
          x.nu3 = lm[li].nu3;
          x.P2 = lm[li].P2;
        }
      }
    }
    rc |= dupload(&T.ma_down, di.data(), di.size());
    rc |= dupload(&T.ma_up, ui_.data(), ui_.size());
  }
  // macro-atom records per level (engine_dev.h DevCells::ma_rec): recombination targets are the ionising levels
  // of the lower ion for levels l <= maxrecombininglevel of ions i > 0 (macroatom.cc:104-124); up-higher targets
  // are the phixs targets of ionising levels of non-top ions (get_nphixstargets)
  std::vector<MaMeta> mm(nl);
  std::vector<int64_t> dbl_off(nl + 1, 0);  // exact-sum scratch of k_marates (doubles, unpadded)
  int64_t marec = 0;
  bool ma_cache_ok = true;  // every level's same-ion arrays fit the two-level record layout
  for (int e = 0; e < ne; e++)
    for (int i = 0; i < a->elem_nions[e]; i++) {
      const int ui = a->elem_uniqueionoffset[e] + i;
      for (int l = 0; l < a->ion_nlevels[ui]; l++) {
        const int ul = a->ion_uniqueleveloffset[ui] + l;
        MaMeta &m = mm[ul];
        m.nr = (i > 0 && l <= a->ion_maxrecombininglevel[ui]) ? a->ion_ionisinglevels[ui - 1] : 0;
        m.nt = (i < a->elem_nions[e] - 1 && l < a->ion_ionisinglevels[ui]) ? a->level_nphixstargets[ul] : 0;
        m.nd = a->level_ndowntrans[ul];
        m.nu = a->level_nuptrans[ul];
        m.doff = a->level_downtrans_offset[ul];
        m.uoff = a->level_uptrans_offset[ul];
        m.base_lower = (i > 0) ? a->ion_uniqueleveloffset[ui - 1] : -1;
        m.rec_off = (int32_t)marec;
        const int64_t len = ARTIS_MA_ACTION_COUNT + 2 * (int64_t)m.nd + m.nu + 2 * (int64_t)m.nr + m.nt;
        // high then low key halves (engine_dev.h ma_layout), records 128-byte aligned
        marec += (2 * (int64_t)ma_layout(m.nd, m.nu, m.nr, m.nt).hot + 63) / 64 * 64;
        dbl_off[ul + 1] = len;
        if (!ma_layout_ok(m.nd, m.nu)) ma_cache_ok = false;
      }
    }
  rc |= dupload(&T.ma_meta, mm.data(), nl);
  {
    std::vector<MaWalk> mw(nl);
    for (int ul = 0; ul < nl; ul++)
      if (!ma_walk_make(mm[ul], &mw[ul])) ma_cache_ok = false;
    rc |= dupload(&T.ma_walk, mw.data(), nl);
  }
  for (int ul = 0; ul < nl; ul++) dbl_off[ul + 1] += dbl_off[ul];
  rc |= dupload(&T.ma_dbl_off, dbl_off.data(), nl + 1);
  G.h_dbl_off = dbl_off;
  {
    // internal same-ion jump targets in the (reference) order of their cumulative arrays
    std::vector<int2> dt(std::max<int64_t>(ndown, 1)), ut(std::max<int64_t>(nup, 1));
    for (int e = 0; e < ne; e++)
      for (int i = 0; i < a->elem_nions[e]; i++) {
        const int ui = a->elem_uniqueionoffset[e] + i;
        const int base = a->ion_uniqueleveloffset[ui];
        for (int l = 0; l < a->ion_nlevels[ui]; l++) {
          const int ul = base + l;
          const MaMeta &m = mm[ul];
          for (int j = 0; j < m.nd; j++) {
            const int t = base + a->line_lowerlevelindex[a->downtrans_lineindex[m.doff + j]];
            dt[m.doff + j] = make_int2(t, mm[t].rec_off);
          }
          for (int j = 0; j < m.nu; j++) {
            const int t = base + a->line_upperlevelindex[a->uptrans_lineindex[m.uoff + j]];
            ut[m.uoff + j] = make_int2(t, mm[t].rec_off);
          }
        }
      }
    rc |= dupload(&T.down_target, dt.data(), dt.size());
    rc |= dupload(&T.up_target, ut.data(), ut.size());
  }
  G.ma_key_stride = marec;
  G.ma_cache_ok = ma_cache_ok;
  rc |= dupload(&T.allcont_nu_edge, a->allcont_nu_edge, nb);
  rc |= dupload(&T.allcont_probability, a->allcont_probability, nb);
  rc |= dupload(&T.allcont_element, a->allcont_element, nb);
  rc |= dupload(&T.allcont_ion, a->allcont_ion, nb);
  rc |= dupload(&T.allcont_level, a->allcont_level, nb);
  rc |= dupload(&T.allcont_target, a->allcont_phixstargetindex, nb);
  rc |= dupload(&T.allcont_upperlevel, a->allcont_upperlevel, nb);
  rc |= dupload(&T.allcont_phixstable, a->allcont_phixstable, nb);
  {
    std::vector<BfCont> bc(std::max(1, nb));
    for (int i = 0; i < nb; i++) {
      bc[i].nu_edge = a->allcont_nu_edge[i];
      bc[i].nu_max = a->allcont_nu_edge[i] * a->last_phixs_nuovernuedge;  // (bf_contribution's expression)
      bc[i].probability = a->allcont_probability[i];
      bc[i].xs_off = a->allcont_phixstable[i] * a->nphixspoints;
      bc[i].pad = 0;
    }
    rc |= dupload(&T.bfc, bc.data(), bc.size());
    const int ne2 = (nb / 4 + 1) * 4;  // at least one padding entry
    std::vector<double2> e2(ne2, make_double2(INFINITY, INFINITY));
    for (int i = 0; i < nb; i++) e2[i] = make_double2(bc[i].nu_edge, bc[i].nu_max);
    rc |= dupload(&T.bf_edge2, e2.data(), e2.size());
  }
  rc |= dupload(&T.allcont_groundindex, a->allcont_index_in_groundphixslist, nb);
  rc |= dupload(&T.groundcont_nu_edge, a->groundcont_nu_edge, a->nbfcontinua_ground);
  {
    // per ground continuum, the allcont indices (ascending) of the ground-level continua that enter its
    // groundcont_gamma_contr (rpkt.cc:1166-1171): update_estimators sums these instead of scanning all continua
    const int nbfg = a->nbfcontinua_ground;
    std::vector<int32_t> off(nbfg + 1, 0), lst;
    for (int g = 0; g < nbfg; g++) {
      off[g] = (int32_t)lst.size();
      for (int i = 0; i < nb; i++)
        if (a->allcont_level[i] == 0 && a->allcont_index_in_groundphixslist[i] == g) lst.push_back(i);
    }
    off[nbfg] = (int32_t)lst.size();
    if (lst.empty()) lst.push_back(0);
    rc |= dupload(&T.gc_cont_off, off.data(), off.size());
    rc |= dupload(&T.gc_cont, lst.data(), lst.size());
  }
  rc |= dupload(&T.groundcont_element, a->groundcont_element, a->nbfcontinua_ground);
  rc |= dupload(&T.groundcont_ion, a->groundcont_ion, a->nbfcontinua_ground);
  rc |= dupload(&T.spontrecombcoeff, a->spontrecombcoeff, (size_t)a->tablesize * nb);
  rc |= dupload(&T.corrphotoioncoeff, a->corrphotoioncoeff, (size_t)a->tablesize * nb);
  rc |= dupload(&T.bfcooling_coeff, a->bfcooling_coeff, (size_t)a->tablesize * nb);
  rc |= dupload(&T.cool_type, a->coolinglist_type, a->ncoolingterms);
  rc |= dupload(&T.cool_element, a->coolinglist_element, a->ncoolingterms);
  rc |= dupload(&T.cool_ion, a->coolinglist_ion, a->ncoolingterms);
  rc |= dupload(&T.cool_level, a->coolinglist_level, a->ncoolingterms);
  rc |= dupload(&T.cool_upper, a->coolinglist_upperlevel, a->ncoolingterms);
  // photoionisation target slots -> (unique level, target index)
  std::vector<int32_t> tul(ntg + 1), tt(ntg + 1);
  for (int ul = 0; ul < nl; ul++)
    for (int t = 0; t < a->level_nphixstargets[ul]; t++) {
      tul[a->level_phixstargets_offset[ul] + t] = ul;
      tt[a->level_phixstargets_offset[ul] + t] = t;
    }
  const int32_t *dtul, *dtt;
  rc |= dupload(&dtul, tul.data(), ntg + 1);
  rc |= dupload(&dtt, tt.data(), ntg + 1);
  G.d_target_ul = const_cast<int32_t *>(dtul);
  G.d_target_t = const_cast<int32_t *>(dtt);

  // geometry
  DevGeom &GG = G.K.G;
  for (int d = 0; d < 3; d++) GG.ncoordgrid[d] = g->ncoordgrid[d];
  GG.ngrid = g->ngrid;
  GG.npts_model = g->npts_model;
  rc |= dupload(&GG.cell_pos_min, g->cell_pos_min, (size_t)g->ngrid * 3);
  rc |= dupload(&GG.cell_mgi, g->cell_mgi, g->ngrid);
  GG.spherical = g->grid_type == ARTIS_GRID_SPHERICAL1D;
  GG.cell_wid = nullptr;
  if (GG.spherical) rc |= dupload(&GG.cell_wid, g->modelcell_wid_init, g->ngrid);
  GG.coordmax0 = g->coordmax[0];
  GG.tmin = g->tmin;
  GG.tmax = g->tmax;
  GG.vmax = g->vmax;
  GG.rmax = g->rmax;
  GG.wid = 2 * g->coordmax[0] / g->ncoordgrid[0];  // grid.cc:76-91
  G.ntstep = g->ntstep;
  rc |= dupload(&GG.ts_start, g->ts_start, g->ntstep);
  rc |= dupload(&GG.ts_width, g->ts_width, g->ntstep);
  rc |= dupload(&GG.ts_mid, g->ts_mid, g->ntstep);
  GG.nu_min_r = g->nu_min_r;
  GG.nu_max_r = g->nu_max_r;

  DevRun &R = G.K.R;
  R.seed = rp->seed;
  R.rank = rp->rank;
  R.opacity_case = rp->opacity_case;
  R.do_r_lc = rp->do_r_lc;
  R.do_rlc_est = rp->do_rlc_est;
  R.n_kpktdiffusion_timesteps = rp->n_kpktdiffusion_timesteps;
  R.kpktdiffusion_timescale = rp->kpktdiffusion_timescale;
  R.max_path_step = rp->max_path_step;
  R.pol_dipole = rp->pol_dipole;
  R.relativistic_doppler = rp->relativistic_doppler;
  R.record_linestat = rp->record_linestat;
  R.gamma_grey = rp->gamma_grey;
  R.instant_particle_deposition = rp->instant_particle_deposition;
  R.nt_solve_spencerfano = rp->nt_solve_spencerfano;
  if (rp->excitation_temperature != ARTIS_TEXC_TJ && rp->excitation_temperature != ARTIS_TEXC_TE) {
    G.last_error = "artis_run_params.excitation_temperature must be ARTIS_TEXC_TJ or ARTIS_TEXC_TE";
    return ARTIS_ERR_BAD_ARGUMENT;
  }
  R.exc_te = rp->excitation_temperature == ARTIS_TEXC_TE;
  R.minpop = rp->minpop > 0. ? rp->minpop : 1e-30;
  R.nlte_on = rp->nlte_pops_on;
  R.multibin = rp->multibin_radfield;
  R.first_nlte_rf = rp->first_nlte_radfield_timestep;
  R.detailed_bf = rp->detailed_bf_estimators;
  R.detailed_bf_usefrom = rp->detailed_bf_usefromtimestep;
  R.no_lut_photoion = rp->no_lut_photoion;
  R.no_lut_bfheating = rp->no_lut_bfheating;
  R.nt_on = rp->nt_on;
  R.nt_max_auger = rp->nt_max_auger_electrons;
  R.nts = -1;
  R.comp_est = rp->comp_est;
  R.comp_est_now = 0;
  R.emiss_offset = rp->emiss_offset;
  R.emiss_max = rp->emiss_max;
  R.time_syn_first = rp->time_syn_first;
  R.time_syn_last = rp->time_syn_last;
  for (int d = 0; d < 3; d++) R.syn_dir[d] = rp->syn_dir[d];
  if (R.comp_est && (R.emiss_max < 1 || R.emiss_max > ARTIS_EMISS_MAX)) {
    G.last_error = "artis_run_params.emiss_max must be in [1, ARTIS_EMISS_MAX] with comp_est (input.cc:1821-1824)";
    return ARTIS_ERR_BAD_ARGUMENT;
  }
  if ((R.nlte_on && (!a->ion_nlevels_nlte || !a->ion_first_nlte || a->total_nlte_levels < 0)) ||
      (R.multibin && (a->radfield_nbins <= 0 || !a->radfield_nu_upper)) || R.nt_max_auger < 0) {
    G.last_error = "nebular run parameters without the atomic tables they need (ion_nlevels_nlte / radfield bins)";
    return ARTIS_ERR_BAD_ARGUMENT;
  }
  T.total_nlte_levels = R.nlte_on ? a->total_nlte_levels : 0;
  T.rf_nbins = R.multibin ? a->radfield_nbins : 0;
  T.rf_nu_lower_first = a->radfield_nu_lower_first;
  if (R.nlte_on) {
    rc |= dupload(&T.ion_nlevels_nlte, a->ion_nlevels_nlte, ni);
    rc |= dupload(&T.ion_first_nlte, a->ion_first_nlte, ni);
  }
  if (R.multibin) rc |= dupload(&T.rf_nu_upper, a->radfield_nu_upper, a->radfield_nbins);
  {
    // get_bfcontindex (radfield.cc:1329-1341): the allcont entry of each photoionisation target slot
    std::vector<int32_t> sa(ntg + 1, -1);
    for (int ib = 0; ib < nb; ib++) {
      const int ul = a->ion_uniqueleveloffset[a->elem_uniqueionoffset[a->allcont_element[ib]] + a->allcont_ion[ib]] +
                     a->allcont_level[ib];
      sa[a->level_phixstargets_offset[ul] + a->allcont_phixstargetindex[ib]] = ib;
    }
    rc |= dupload(&T.slot_allcont, sa.data(), ntg + 1);
    // bflist (input.cc:1153-1160: cont_index counts down from -1 over every level's targets) -> ion column
    std::vector<int32_t> bc(std::max(nb, 1), 0);
    for (int e = 0; e < ne; e++)
      for (int i = 0; i < a->elem_nions[e]; i++) {
        const int ui = a->elem_uniqueionoffset[e] + i;
        for (int l = 0; l < a->ion_nlevels[ui]; l++) {
          const int ul = a->ion_uniqueleveloffset[ui] + l;
          for (int t = 0; t < a->level_nphixstargets[ul]; t++) {
            const int bi = -1 - (a->level_cont_index[ul] - t);
            if (bi >= 0 && bi < nb) bc[bi] = e * a->maxnions + i;
          }
        }
      }
    const int32_t *dbc;
    rc |= dupload(&dbc, bc.data(), bc.size());
    G.d_bfcol = const_cast<int32_t *>(dbc);
  }

  // estimators: one double block [J | nuJ | ffheat | colheat | rpkt_emiss | gamma | bfheat | scalars(10) |
  // bfrate_raw | radfield J_raw | nuJ_raw | contribcount | compton_emiss] (the nebular sections only when their
  // option is on)
  const int np = g->npts_model;
  const int64_t nion_est = (int64_t)np * ne * a->maxnions;
  G.nbf_est = R.detailed_bf ? nb : 0;
  G.nbins_est = T.rf_nbins;
  G.n_est_doubles = 5 * (int64_t)np + 2 * nion_est + 10 + (int64_t)np * (G.nbf_est + 3 * G.nbins_est) +
                    ((int64_t)np + 1) * ARTIS_EMISS_MAX;
  rc |= dalloc(&G.d_estblock, G.n_est_doubles);
  DevEst &E = G.K.E;
  E.J = G.d_estblock;
  E.nuJ = E.J + np;
  E.ffheat = E.nuJ + np;
  E.colheat = E.ffheat + np;
  E.rpkt_emiss = E.colheat + np;
  E.gamma = E.rpkt_emiss + np;
  E.bfheat = E.gamma + nion_est;
  E.scalars = E.bfheat + nion_est;
  E.bfrate = E.scalars + 10;
  E.rfJ = E.bfrate + (int64_t)np * G.nbf_est;
  E.rfnuJ = E.rfJ + (int64_t)np * G.nbins_est;
  E.rfcount = E.rfnuJ + (int64_t)np * G.nbins_est;
  E.compton = E.rfcount + (int64_t)np * G.nbins_est;
  rc |= dalloc(&E.ecounter, nli);
  rc |= dalloc(&E.acounter, nli);
  rc |= dalloc(&E.counters, ARTIS_COUNTER_COUNT + 1);
  rc |= dalloc(&E.work, ARTIS_WORK_COUNT);
  rc |= dalloc(&E.err, 4);
  if (rc) return ARTIS_ERR_HIP;
  G.npts_model = np;
  G.nelements = ne;
  G.maxnions = a->maxnions;
  G.nions_total = ni;
  G.nlines = nli;
  G.ngrid = g->ngrid;
  // non-empty model cells: those referenced by a propagation cell, numbered from the centre outwards (the
  // distance of the cell's nearest propagation-cell centre at tmin, ties by mgi) -- the per-cell tables that only
  // fit the HBM budget for some cells (line coefficients, macro-atom keys) hold the first rows, the cells where
  // the packets start and the density peaks; every other cell takes the equivalent table-free path
  std::vector<int32_t> ne_index(np, -1), ne_mgi;
  std::vector<double> rmin(np, DBL_MAX);
  for (int c = 0; c < g->ngrid; c++) {
    const int mgi = g->cell_mgi[c];
    if (mgi >= 0 && mgi < np) {
      double r2 = 0.;
      if (g->grid_type == ARTIS_GRID_SPHERICAL1D) {
        const double r = g->cell_pos_min[3 * (int64_t)c] + 0.5 * g->modelcell_wid_init[c];  // get_cellradialpos
        r2 = r * r;
      } else {
        for (int d = 0; d < 3; d++) {
          const double x = g->cell_pos_min[3 * (int64_t)c + d] + g->coordmax[d] / std::max(1, g->ncoordgrid[d]);
          r2 += x * x;
        }
      }
      rmin[mgi] = std::min(rmin[mgi], r2);
      ne_index[mgi] = 0;
    }
  }
  for (int mgi = 0; mgi < np; mgi++)
    if (ne_index[mgi] == 0) ne_mgi.push_back(mgi);
  std::stable_sort(ne_mgi.begin(), ne_mgi.end(), [&](int a, int b) { return rmin[a] < rmin[b]; });
  for (size_t k = 0; k < ne_mgi.size(); k++) ne_index[ne_mgi[k]] = (int32_t)k;
  const int nne_cells = (int)ne_mgi.size();
  const int32_t *dnei, *dnem;
  rc |= dupload(&dnei, ne_index.data(), np);
  rc |= dupload(&dnem, ne_mgi.data(), nne_cells);
  DevCells &C = G.K.C;
  C.ne_index = dnei;
  C.ne_mgi = dnem;
  C.n_nonempty = nne_cells;
  {
    // few-cell models: k_rpkt accumulates the estimators of every non-empty cell per block in LDS, as many of the
    // sections as fit (ARTIS_GPU_NO_EST_LDS=1: none)
    const char *ne = getenv("ARTIS_GPU_NO_EST_LDS");
    const bool allow = !(ne && ne[0] == '1');
    int64_t off = 0;
    auto take = [&](bool want, int64_t n) -> int32_t {
      if (!allow || !want || n <= 0 || off + n > EST_LDS_DOUBLES) return -1;
      const int32_t o = (int32_t)off;
      off += n;
      return o;
    };
    C.est_lds_J = take(true, 3 * (int64_t)nne_cells);
    C.est_lds_bf = take(G.K.R.detailed_bf != 0, (int64_t)nne_cells * G.K.T.nbf);
    C.est_lds_rf = take(G.K.R.multibin != 0, 3 * (int64_t)nne_cells * G.K.T.rf_nbins);
  }
  rc |= dalloc(&G.W.bins, (size_t)nne_cells + 1);
  rc |= dalloc(&G.d_binoffs, (size_t)nne_cells + 1);
  rc |= dalloc(&G.W.xhead, (size_t)8);
  if (!rc) {
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, G.scan_tmp_bytes, G.W.bins, G.d_binoffs, nne_cells + 1);
    rc |= dalloc((char **)&G.d_scan_tmp, G.scan_tmp_bytes);
  }
  rc |= dalloc(&C.pops, (size_t)nne_cells * nl);
  rc |= dalloc(&C.ionpop, (size_t)nne_cells * ni);
  rc |= dalloc(&C.ffsum, (size_t)nne_cells);
  rc |= dalloc(&C.bfcell, (size_t)nne_cells * nb);
  rc |= dalloc(&C.corrphot, (size_t)nne_cells * (ntg + 1));
  rc |= dalloc(&C.popsT, (size_t)nne_cells * nl);
  rc |= dalloc(&C.corrphotT, (size_t)nne_cells * (ntg + 1));
  rc |= dalloc(&C.cooling, (size_t)nne_cells * a->ncoolingterms);
  C.ma_key_stride = G.ma_key_stride;
  C.have_macache = 0;
  C.ma_rows = 0;
  C.ma_key = nullptr;
  C.marates = nullptr;
  C.ma_lptr = nullptr;
  C.ma_lhist = nullptr;
  C.ma_level_mode = 0;
  C.ma_hi_only = 0;
  {
    // Macro-atom key records.  Row mode when every non-empty cell's records fit the budget (default: half of the
    // free HBM, ARTIS_GPU_MACACHE_MAX_GB; the rest is left for the packet store): cell k's records at row k.
    // Otherwise level mode: a pool of (cell, level) records within the same budget, less the per-pair action
    // totals the walks without a record read (k_ma's cooperative jump) and the pointer / activity tables; the
    // records go to the pairs the walks used most in the previous timestep (ma_level_place).
    // ARTIS_GPU_MACACHE_ROWS=r (tests) caps the budget at r rows' worth; ARTIS_GPU_NO_MACACHE=1 leaves the pool
    // empty (every jump cooperative, exact sums).  The split never changes a result.
    size_t freeb = 0, totalb = 0;
    (void)hipMemGetInfo(&freeb, &totalb);
    const double row_bytes = (double)C.ma_key_stride * 2.0;
    int64_t maxlev = 0;
    for (int ul = 0; ul < nl; ul++) maxlev = std::max(maxlev, G.h_dbl_off[ul + 1] - G.h_dbl_off[ul]);
    int64_t cap = ((int64_t)2 << 30) / 8;  // k_marates scratch of row mode (ARTIS_GPU_MAREC_SCRATCH_MB)
    if (const char *sm = getenv("ARTIS_GPU_MAREC_SCRATCH_MB")) cap = (int64_t)(atof(sm) * (1 << 20) / 8);
    const int64_t scratch = std::max<int64_t>(maxlev * MARATES_PAD(nne_cells),
                                              std::min<int64_t>(G.h_dbl_off[nl] * MARATES_PAD(nne_cells), cap));
    double budget = 0.5 * (double)freeb;
    if (const char *mx = getenv("ARTIS_GPU_MACACHE_MAX_GB")) budget = atof(mx) * (double)(1ull << 30);
    const char *mr = getenv("ARTIS_GPU_MACACHE_ROWS");
    if (mr) budget = std::min(budget, (double)atoll(mr) * row_bytes);
    const char *env = getenv("ARTIS_GPU_NO_MACACHE");
    const bool none = env && env[0] == '1';
    const bool rows_fit = !none && G.ma_cache_ok &&
                          (double)nne_cells * row_bytes + 8.0 * (double)scratch <= budget &&
                          (double)nne_cells * row_bytes / 128.0 < 4.0e9;
    void *mc = nullptr, *sc = nullptr;
    if (rows_fit && dmalloc(&mc, (size_t)((double)nne_cells * row_bytes)) == hipSuccess) {
      G.allocs.push_back(mc);
      if (dmalloc(&sc, (size_t)scratch * 8) == hipSuccess) {
        G.allocs.push_back(sc);
        C.ma_key = (uint16_t *)mc;
        C.have_macache = 1;
        C.ma_rows = nne_cells;
        G.d_marec_scratch = (double *)sc;
        G.marec_scratch_doubles = scratch;
      }
    }
    if (!C.ma_rows) {
      // level mode: per level, its record size in 128-byte lines (0: never a record -- a layout that does not fit,
      // or more rate terms than k_ma_build stages in LDS)
      G.h_rec_lines.assign(nl, 0);
      G.ma_build_lds_doubles = 0;
      const bool hi_only = ARTIS_MA_HI_ONLY;  // (k_ma's level-mode instance compiles the same choice in)
      std::vector<MaMeta> mm(nl);
      HIPCHK(hipMemcpy(mm.data(), G.K.T.ma_meta, nl * sizeof(MaMeta), hipMemcpyDeviceToHost));
      for (int ul = 0; ul < nl; ul++) {
        const int64_t next = (ul + 1 < nl) ? mm[ul + 1].rec_off : G.ma_key_stride;
        const int64_t need = ma_build_doubles(mm[ul]);
        if (ma_layout_ok(mm[ul].nd, mm[ul].nu) && need <= MA_BUILD_MAX_DOUBLES) {
          const int64_t hot = ma_layout(mm[ul].nd, mm[ul].nu, mm[ul].nr, mm[ul].nt).hot;
          G.h_rec_lines[ul] = (uint32_t)(hi_only ? (hot + 63) / 64 : (next - mm[ul].rec_off) / 64);
          G.ma_build_lds_doubles = std::max<int64_t>(G.ma_build_lds_doubles, need);
        }
      }
      const double tables = (double)nne_cells * nl * (ARTIS_MA_ACTION_COUNT * 8.0 + 8.0);
      // (ARTIS_GPU_MACACHE_ROWS: a pool of exactly that many rows' records)
      const double pool = none ? 128.0 : mr ? std::max(128.0, budget) : std::max(128.0, budget - tables);
      G.ma_pool_lines = (uint64_t)std::min(pool / 128.0, 4.0e9 - 1.0);
      if (dmalloc(&mc, (size_t)G.ma_pool_lines * 128) == hipSuccess) {
        G.allocs.push_back(mc);
        C.ma_key = (uint16_t *)mc;
        C.have_macache = 1;
        C.ma_level_mode = 1;
        C.ma_hi_only = hi_only ? 1 : 0;
        rc |= dalloc(&C.marates, (size_t)nne_cells * nl * ARTIS_MA_ACTION_COUNT);
        rc |= dalloc(&G.d_ma_lptr, (size_t)nne_cells * nl);
        rc |= dalloc(&G.d_ma_lhist, (size_t)nne_cells * nl);
        rc |= dupload(&G.d_rec_lines, G.h_rec_lines.data(), nl);
        std::vector<uint32_t> rl_off(nl, 0);
        uint64_t acc = 0;
        for (int ul = 0; ul < nl; ul++) {
          rl_off[ul] = (uint32_t)acc;
          acc += G.h_rec_lines[ul];
        }
        G.row_lines = (uint32_t)acc;
        rc |= dupload(&G.d_rl_off, rl_off.data(), nl);
        rc |= dalloc(&G.d_lvl_ctr, (size_t)4);
        rc |= dalloc(&G.d_lvl_buckets, (size_t)(2 + MA_LVL_NB));
        rc |= dalloc(&G.d_build_list, (size_t)std::max<int64_t>(1, std::min<int64_t>((int64_t)nne_cells * nl,
                                                                                   (int64_t)G.ma_pool_lines)));
        G.build_list_cap = std::min<int64_t>((int64_t)nne_cells * nl, (int64_t)G.ma_pool_lines);
        C.ma_lptr = G.d_ma_lptr;
        C.ma_lhist = G.d_ma_lhist;
        G.ma_lhist_ready = false;
      } else {
        rc |= ARTIS_ERR_HIP;
      }
    }
  }
  rc |= dalloc(&G.d_ma_row, (size_t)nne_cells);
  rc |= dalloc(&G.d_ma_bin, (size_t)nne_cells);
  rc |= dalloc(&G.d_ma_bincell, (size_t)nne_cells);
  C.ma_row = G.d_ma_row;
  C.ma_bin = G.d_ma_bin;
  if (!rc) {
    std::vector<int32_t> order(nne_cells);
    for (int k = 0; k < nne_cells; k++) order[k] = k;  // centre outwards
    rc |= ma_place(order);
  }
  // per-cell line coefficients for the r-packet line walk: rows for the first linecoef_rows cells (centre
  // outwards) within a budget of 30% of the HBM still free (the packet store comes later; ARTIS_GPU_LINECOEF_MAX_GB
  // overrides it), ARTIS_GPU_NO_LINECOEF=1 switches them off.  Cells past the last row gather the two populations
  // per line themselves (the same coefficient, bit for bit).
  C.linecoef = nullptr;
  C.linecoef_rows = 0;
  C.linecoef_stride = ((int64_t)G.K.T.nlines + 15) / 16 * 16;  // (whole 16-line windows: k_vpkt)
  {
    size_t freeb = 0, totalb = 0;
    (void)hipMemGetInfo(&freeb, &totalb);
    double budget = 0.3 * (double)freeb;
    if (const char *mx = getenv("ARTIS_GPU_LINECOEF_MAX_GB")) budget = atof(mx) * (double)(1ull << 30);
    const char *env = getenv("ARTIS_GPU_NO_LINECOEF");
    const double row_bytes = (double)C.linecoef_stride * 8.0;
    int rows = (int)std::min<double>((double)nne_cells, std::floor(budget / row_bytes));
    if (const char *lr = getenv("ARTIS_GPU_LINECOEF_ROWS")) rows = std::min(rows, atoi(lr));
    if (env && env[0] == '1') rows = 0;
    if (rows > 0) {
      void *lc = nullptr;
      if (dmalloc(&lc, (size_t)rows * (size_t)row_bytes) == hipSuccess) {
        G.allocs.push_back(lc);
        C.linecoef = (double *)lc;
        C.linecoef_rows = rows;
      }
    }
  }
  C.linecoef_neg = nullptr;
  rc |= dalloc(&C.linecoef_neg, (size_t)1);
  if (C.linecoef_neg) HIPCHK(hipMemset(C.linecoef_neg, 0, sizeof(int32_t)));
  // cell-state input buffers
  rc |= dalloc(&G.W.ctr, (size_t)NQUEUES * 2);
  rc |= dalloc(&G.d_ctx, (size_t)1);
  rc |= dalloc(&G.W.stats, (size_t)48);
  rc |= dalloc(&G.d_cellf, (size_t)9 * np);
  rc |= dalloc(&G.d_thick, (size_t)np);
  rc |= dalloc(&G.d_abund, (size_t)np * ne);
  rc |= dalloc(&G.d_glp, (size_t)np * ni);
  rc |= dalloc(&G.d_pf, (size_t)np * ni);
  rc |= dalloc(&G.d_totcool, (size_t)np);
  rc |= dalloc(&G.d_ccion, (size_t)np * ni);
  rc |= dalloc(&G.d_renorm, (size_t)np * ne * a->maxnions);
  if (R.nlte_on) rc |= dalloc(&G.d_nltepops, (size_t)np * std::max(1, T.total_nlte_levels));
  if (R.multibin) {
    rc |= dalloc(&G.d_rfTR, (size_t)np * T.rf_nbins);
    rc |= dalloc(&G.d_rfW, (size_t)np * T.rf_nbins);
  }
  if (R.detailed_bf) rc |= dalloc(&G.d_bfest, (size_t)np * std::max(1, nb));
  if (R.nt_on) {
    const size_t na = (size_t)R.nt_max_auger + 1;
    rc |= dalloc(&G.d_ntdep, (size_t)np);
    rc |= dalloc(&G.d_ntY, (size_t)np * ni);
    rc |= dalloc(&G.d_ntprob, (size_t)np * ni * na);
    rc |= dalloc(&G.d_ntionen, (size_t)np * ni * na);
    rc |= dalloc(&C.nt_cum, (size_t)std::max(1, nne_cells) * ni);
    rc |= dalloc(&C.nt_total, (size_t)std::max(1, nne_cells));
  }
  if (R.no_lut_photoion && nne_cells > 0 && ntg > 0) {
    // one integration workspace of GSLWSIZE intervals per resident wave of k_corrphot_integral (48 B each)
    G.qag_waves = (int)std::min<int64_t>((int64_t)nne_cells * ntg, 512);
    const size_t nw = (size_t)G.qag_waves * QAG_LIMIT;
    rc |= dalloc(&G.qag.alist, nw);
    rc |= dalloc(&G.qag.blist, nw);
    rc |= dalloc(&G.qag.rlist, nw);
    rc |= dalloc(&G.qag.elist, nw);
    rc |= dalloc(&G.qag.order, nw);
    rc |= dalloc(&G.qag.level, nw);
  }
  if (rc) return ARTIS_ERR_HIP;
  C.nlte_pops = G.d_nltepops;
  C.rf_TR = G.d_rfTR;
  C.rf_W = G.d_rfW;
  C.bfrate_est = G.d_bfest;
  C.nt_dep = G.d_ntdep;
  C.nt_Y = G.d_ntY;
  C.nt_prob = G.d_ntprob;
  C.nt_ionen = G.d_ntionen;
  C.Te = G.d_cellf;
  C.TR = G.d_cellf + np;
  C.TJ = G.d_cellf + 2 * np;
  C.W = G.d_cellf + 3 * np;
  C.nne = G.d_cellf + 4 * np;
  C.nnetot = G.d_cellf + 5 * np;
  C.rho = G.d_cellf + 6 * np;
  C.kappagrey = G.d_cellf + 7 * np;
  C.ffegrp = G.d_cellf + 8 * np;
  C.thick = G.d_thick;
  C.elem_abundance = G.d_abund;
  C.groundlevelpop = G.d_glp;
  C.partfunct = G.d_pf;
  C.totalcooling = G.d_totcool;
  C.cooling_contrib_ion = G.d_ccion;
  C.corrphotoionrenorm = G.d_renorm;
  G.initialised = true;
  return 0;
}

int artis_gpu_init_gamma(const artis_gamma_spectra *gs) {
  if (!G.initialised) return ARTIS_ERR_NOT_INITIALISED;
  if (!gs || gs->nnuclides <= 0 || !gs->nuc_nlines || !gs->nuc_line_offset || !gs->nuc_endecay_gamma) {
    G.last_error = "init_gamma: bad gamma spectra";
    return ARTIS_ERR_BAD_ARGUMENT;
  }
  const int nn = gs->nnuclides;
  int64_t nlines = 0;
  for (int k = 0; k < nn; k++) {
    if (gs->nuc_nlines[k] < 0 || gs->nuc_line_offset[k] < 0) return ARTIS_ERR_BAD_ARGUMENT;
    nlines = std::max<int64_t>(nlines, (int64_t)gs->nuc_line_offset[k] + gs->nuc_nlines[k]);
  }
  if (nlines > 0 && (!gs->line_energy || !gs->line_probability)) return ARTIS_ERR_BAD_ARGUMENT;
  DevTab &T = G.K.T;
  int32_t *nl = nullptr, *off = nullptr;
  double *en = nullptr, *eg = nullptr, *pr = nullptr;
  int rc = 0;
  rc |= dalloc(&nl, (size_t)nn);
  rc |= dalloc(&off, (size_t)nn);
  rc |= dalloc(&eg, (size_t)nn);
  rc |= dalloc(&en, (size_t)std::max<int64_t>(nlines, 1));
  rc |= dalloc(&pr, (size_t)std::max<int64_t>(nlines, 1));
  if (rc) return ARTIS_ERR_HIP;
  HIPCHK(hipMemcpy(nl, gs->nuc_nlines, sizeof(int32_t) * nn, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(off, gs->nuc_line_offset, sizeof(int32_t) * nn, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(eg, gs->nuc_endecay_gamma, sizeof(double) * nn, hipMemcpyHostToDevice));
  if (nlines > 0) {
    HIPCHK(hipMemcpy(en, gs->line_energy, sizeof(double) * nlines, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(pr, gs->line_probability, sizeof(double) * nlines, hipMemcpyHostToDevice));
  }
  T.g_nnuc = nn;
  T.g_nlines = nl;
  T.g_off = off;
  T.g_endecay = eg;
  T.g_energy = en;
  T.g_prob = pr;
  // allnuc_gamma_line_list: every nuclide's lines sorted by energy (init_gamma_linelist, gammapkt.cc:192-211); the
  // Compton emissivity bins by get_nul over its frequencies (gammapkt.cc:720-745)
  std::vector<double> fs;
  for (int k = 0; k < nn; k++)
    for (int j = 0; j < gs->nuc_nlines[k]; j++) fs.push_back(gs->line_energy[gs->nuc_line_offset[k] + j]);
  std::sort(fs.begin(), fs.end());
  for (double &f : fs) f /= ARTIS_H;
  T.g_nsorted = (int32_t)fs.size();
  if (!fs.empty()) {
    const double *dfs;
    rc |= dupload(&dfs, fs.data(), fs.size());
    if (rc) return ARTIS_ERR_HIP;
    T.g_freq_sorted = dfs;
  }
  return 0;
}

int artis_gpu_upload_cellstate(int nts, const artis_cell_state *cs) {
  if (!G.initialised) return ARTIS_ERR_NOT_INITIALISED;
  if (!cs || nts < 0 || nts >= G.ntstep) {
    G.last_error = "upload_cellstate: bad cell state pointer or timestep out of range";
    return ARTIS_ERR_BAD_ARGUMENT;
  }
  const int np = G.npts_model, ne = G.nelements, ni = G.nions_total;
  const float *fsrc[8] = {cs->Te, cs->TR, cs->TJ, cs->W, cs->nne, cs->nnetot, cs->rho, cs->kappagrey};
  for (int f = 0; f < 8; f++)
    HIPCHK(hipMemcpyAsync(G.d_cellf + (size_t)f * np, fsrc[f], sizeof(float) * np, hipMemcpyHostToDevice, G.stream));
  if (cs->ffegrp)
    HIPCHK(hipMemcpyAsync(G.d_cellf + (size_t)8 * np, cs->ffegrp, sizeof(float) * np, hipMemcpyHostToDevice, G.stream));
  else
    HIPCHK(hipMemsetAsync(G.d_cellf + (size_t)8 * np, 0, sizeof(float) * np, G.stream));
  HIPCHK(hipMemcpyAsync(G.d_thick, cs->thick, sizeof(int16_t) * np, hipMemcpyHostToDevice, G.stream));
  HIPCHK(hipMemcpyAsync(G.d_abund, cs->elem_abundance, sizeof(float) * np * ne, hipMemcpyHostToDevice, G.stream));
  HIPCHK(hipMemcpyAsync(G.d_glp, cs->groundlevelpop, sizeof(float) * np * ni, hipMemcpyHostToDevice, G.stream));
  HIPCHK(hipMemcpyAsync(G.d_pf, cs->partfunct, sizeof(float) * np * ni, hipMemcpyHostToDevice, G.stream));
  HIPCHK(hipMemcpyAsync(G.d_totcool, cs->totalcooling, sizeof(double) * np, hipMemcpyHostToDevice, G.stream));
  HIPCHK(hipMemcpyAsync(G.d_ccion, cs->cooling_contrib_ion, sizeof(double) * np * ni, hipMemcpyHostToDevice, G.stream));
  HIPCHK(hipMemcpyAsync(G.d_renorm, cs->corrphotoionrenorm, sizeof(double) * np * ne * G.maxnions,
                        hipMemcpyHostToDevice, G.stream));
  {
    // the nebular inputs (ABI 6) of the options switched on
    const DevRun &R = G.K.R;
    const int nb = G.K.T.nbf, nbins = G.K.T.rf_nbins;
    const size_t na = (size_t)R.nt_max_auger + 1;
    if ((R.nlte_on && !cs->nlte_pops) || (R.multibin && (!cs->radfield_bin_TR || !cs->radfield_bin_W)) ||
        (R.detailed_bf && !cs->bfrate_estimator) || (R.nt_on && !cs->nt_ionization_ratecoeff) ||
        (R.nt_on && R.nt_solve_spencerfano &&
         (!cs->nt_deposition_rate_density || (R.nt_max_auger > 0 && (!cs->nt_prob_num_auger || !cs->nt_ionenfrac_num_auger))))) {
      G.last_error = "upload_cellstate: a nebular option is on but its cell-state array is NULL";
      return ARTIS_ERR_BAD_ARGUMENT;
    }
    if (R.nlte_on && G.K.T.total_nlte_levels > 0)
      HIPCHK(hipMemcpyAsync(G.d_nltepops, cs->nlte_pops, sizeof(double) * np * G.K.T.total_nlte_levels,
                            hipMemcpyHostToDevice, G.stream));
    if (R.multibin) {
      HIPCHK(hipMemcpyAsync(G.d_rfTR, cs->radfield_bin_TR, sizeof(float) * np * nbins, hipMemcpyHostToDevice, G.stream));
      HIPCHK(hipMemcpyAsync(G.d_rfW, cs->radfield_bin_W, sizeof(float) * np * nbins, hipMemcpyHostToDevice, G.stream));
    }
    if (R.detailed_bf && nb > 0)
      HIPCHK(hipMemcpyAsync(G.d_bfest, cs->bfrate_estimator, sizeof(float) * np * nb, hipMemcpyHostToDevice, G.stream));
    if (R.nt_on) {
      HIPCHK(hipMemcpyAsync(G.d_ntY, cs->nt_ionization_ratecoeff, sizeof(double) * np * ni, hipMemcpyHostToDevice,
                            G.stream));
      if (cs->nt_deposition_rate_density)
        HIPCHK(hipMemcpyAsync(G.d_ntdep, cs->nt_deposition_rate_density, sizeof(double) * np, hipMemcpyHostToDevice,
                              G.stream));
      if (cs->nt_prob_num_auger && cs->nt_ionenfrac_num_auger) {
        HIPCHK(hipMemcpyAsync(G.d_ntprob, cs->nt_prob_num_auger, sizeof(float) * np * ni * na, hipMemcpyHostToDevice,
                              G.stream));
        HIPCHK(hipMemcpyAsync(G.d_ntionen, cs->nt_ionenfrac_num_auger, sizeof(float) * np * ni * na,
                              hipMemcpyHostToDevice, G.stream));
      }
    }
  }
  G.K.R.nts = nts;
  HIPCHK(hipStreamSynchronize(G.stream));
  if (G.K.C.ma_level_mode)
    if (int rc = ma_level_place()) return rc;
  HIPCHK(hipMemsetAsync(G.K.E.err, 0, 4 * sizeof(int32_t), G.stream));
  const int n_ne = G.K.C.n_nonempty;
  const int64_t nl = G.K.T.nlevels_total;
  HIPCHK(hipEventRecord(G.ev0, G.stream));
  if (n_ne > 0) {
    const int B = 256;
    k_cellprep<<<(n_ne + B - 1) / B, B, 0, G.stream>>>(G.K);
    const int64_t nlv = (int64_t)n_ne * nl;
    k_levelpops<<<(unsigned)((nlv + B - 1) / B), B, 0, G.stream>>>(G.K);
    const int64_t nbt = (int64_t)n_ne * (G.K.T.nbf + G.K.T.ntargets_total);
    k_bfcells<<<(unsigned)((nbt + B - 1) / B), B, 0, G.stream>>>(G.K, G.d_target_ul, G.d_target_t);
    if (G.K.R.no_lut_photoion && G.qag_waves > 0)
      k_corrphot_integral<<<(unsigned)G.qag_waves, 64, 0, G.stream>>>(G.K, G.d_target_ul, G.d_target_t, G.qag);
    if (G.K.R.nt_on) k_ntcells<<<(n_ne + B - 1) / B, B, 0, G.stream>>>(G.K);
    k_transpose<<<dim3((unsigned)((nl + 63) / 64), (unsigned)((n_ne + 63) / 64)), 256, 0, G.stream>>>(
        G.K.C.pops, G.K.C.popsT, n_ne, nl);
    const int64_t nci = (int64_t)n_ne * ni;
    k_cooling<<<(unsigned)((nci + 63) / 64), 64, 0, G.stream>>>(G.K);
    const int64_t ntg = G.K.T.ntargets_total;
    if (ntg > 0)
      k_transpose<<<dim3((unsigned)((ntg + 63) / 64), (unsigned)((n_ne + 63) / 64)), 256, 0, G.stream>>>(
          G.K.C.corrphot, G.K.C.corrphotT, n_ne, ntg);
    if (G.K.C.linecoef) HIPCHK(hipMemsetAsync(G.K.C.linecoef_neg, 0, sizeof(int32_t), G.stream));
    if (G.K.C.linecoef) {
      const int lc_rows_lds = (int)std::min<int64_t>(5, LINECOEF_LDS_DOUBLES / std::max<int64_t>(1, nl));
      const char *lcg = getenv("ARTIS_GPU_LINECOEF_GATHER");  // (A/B and test switch: the gather kernel)
      const bool lc_gather = lcg && atoi(lcg);
      if (lc_rows_lds >= 1 && !lc_gather)
        k_linecoef_lds<<<(unsigned)std::min<int64_t>((G.K.C.linecoef_rows + lc_rows_lds - 1) / lc_rows_lds,
                                                     (int64_t)G.wave_grid / 2),  // (4 blocks per CU; one fits)
                         1024, 0, G.stream>>>(G.K, lc_rows_lds);
      else
        k_linecoef<<<dim3((unsigned)((G.K.C.linecoef_stride + 255) / 256),
                          (unsigned)std::min((G.K.C.linecoef_rows + LINECOEF_R - 1) / LINECOEF_R, 32768)), 256, 0,
                      G.stream>>>(G.K);
    }
    const int mr = G.K.C.ma_rows;
    if (G.K.C.ma_level_mode) {
      // level mode: the action totals of every (cell, level) pair (the jumps without a record select from them),
      // then the records the placement chose
      k_marates<false><<<(unsigned)((MARATES_PAD(n_ne) * nl + 255) / 256), 256, 0, G.stream>>>(
          G.K, nts, 0, (int)nl, nullptr, G.d_ma_bincell, n_ne);
      if (int rc = ma_level_build(nts)) return rc;
    } else if (mr > 0) {
      // batches of levels whose records fit the scratch
      for (int ul0 = 0; ul0 < nl;) {
        int ul1 = ul0 + 1;
        while (ul1 < nl && (G.h_dbl_off[ul1 + 1] - G.h_dbl_off[ul0]) * MARATES_PAD(mr) <= G.marec_scratch_doubles) ul1++;
        const int nlev = ul1 - ul0;
        k_marates<true><<<(unsigned)((MARATES_PAD(mr) * nlev + 255) / 256), 256, 0, G.stream>>>(
            G.K, nts, ul0, nlev, G.d_marec_scratch, G.d_ma_bincell, mr);
        k_mapack<<<dim3((unsigned)((mr + 63) / 64), (unsigned)nlev), 256, 0, G.stream>>>(G.K, ul0,
                                                                                         G.d_marec_scratch);
        ul0 = ul1;
      }
    }
    HIPCHK(hipGetLastError());
  }
  HIPCHK(hipEventRecord(G.ev1, G.stream));
  HIPCHK(hipEventSynchronize(G.ev1));
  float ms = 0.f;
  HIPCHK(hipEventElapsedTime(&ms, G.ev0, G.ev1));
  G.last_precompute_ms = ms;
  {
    int32_t neg = 0;
    if (G.K.C.linecoef) HIPCHK(hipMemcpy(&neg, G.K.C.linecoef_neg, sizeof(int32_t), hipMemcpyDeviceToHost));
    G.K.V.neg_coef = neg;
  }
  G.have_cells = true;
  G.cellstate_nts = nts;
  return 0;
}

int artis_gpu_packets_upload(const artis_packet *packets, int npkts) {
  if (!G.initialised) return ARTIS_ERR_NOT_INITIALISED;
  if (npkts < 0 || (npkts > 0 && !packets)) return ARTIS_ERR_BAD_ARGUMENT;
  if (int rc = alloc_packets(npkts)) return rc;
  G.npkts = npkts;
  if (npkts == 0) return 0;
  HIPCHK(hipMemcpyAsync(G.d_aos, packets, (size_t)npkts * sizeof(artis_packet), hipMemcpyHostToDevice, G.stream));
  k_aos_to_soa<<<(unsigned)((npkts + XPOSE_PKTS - 1) / XPOSE_PKTS), 256, 0, G.stream>>>(G.d_aos, G.d_soa, npkts);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(G.stream));
  return 0;
}

int artis_gpu_packets_download(artis_packet *packets, int npkts) {
  if (!G.initialised) return ARTIS_ERR_NOT_INITIALISED;
  if (npkts != G.npkts) return ARTIS_ERR_BAD_ARGUMENT;
  if (npkts == 0) return 0;
  k_soa_to_aos<<<(unsigned)((npkts + XPOSE_PKTS - 1) / XPOSE_PKTS), 256, 0, G.stream>>>(G.d_soa, G.d_aos, npkts);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(packets, G.d_aos, (size_t)npkts * sizeof(artis_packet), hipMemcpyDeviceToHost, G.stream));
  HIPCHK(hipStreamSynchronize(G.stream));
  return 0;
}

int artis_gpu_packets_snapshot(void) {
  if (!G.initialised) return ARTIS_ERR_NOT_INITIALISED;
  if (!G.d_snapshot) HIPCHK(dmalloc((void **)&G.d_snapshot, (size_t)G.cap_pkts * PKT_STORE_WORDS * 8));
  HIPCHK(hipMemcpyAsync(G.d_snapshot, G.d_soa, (size_t)G.npkts * PKT_STORE_WORDS * 8, hipMemcpyDeviceToDevice,
                        G.stream));
  HIPCHK(hipStreamSynchronize(G.stream));
  G.have_snapshot = true;
  return 0;
}

int artis_gpu_packets_restore(void) {
  if (!G.initialised) return ARTIS_ERR_NOT_INITIALISED;
  if (!G.have_snapshot) return ARTIS_ERR_BAD_ARGUMENT;
  HIPCHK(hipMemcpyAsync(G.d_soa, G.d_snapshot, (size_t)G.npkts * PKT_STORE_WORDS * 8, hipMemcpyDeviceToDevice,
                        G.stream));
  return 0;
}

int artis_gpu_estimators_zero(void) {
  if (!G.initialised) return ARTIS_ERR_NOT_INITIALISED;
  const DevEst &E = G.K.E;
  HIPCHK(hipMemsetAsync(G.d_estblock, 0, (size_t)G.n_est_doubles * sizeof(double), G.stream));
  HIPCHK(hipMemsetAsync(E.ecounter, 0, (size_t)G.nlines * sizeof(int32_t), G.stream));
  HIPCHK(hipMemsetAsync(E.acounter, 0, (size_t)G.nlines * sizeof(int32_t), G.stream));
  HIPCHK(hipMemsetAsync(E.counters, 0, (ARTIS_COUNTER_COUNT + 1) * sizeof(unsigned long long), G.stream));
  return 0;
}

int artis_gpu_update_packets_resident(int my_rank, int nts) {
  if (!G.initialised) return ARTIS_ERR_NOT_INITIALISED;
  if (!G.have_cells || G.cellstate_nts != nts) {
    G.last_error = "artis_gpu_upload_cellstate(nts) must precede update_packets(nts)";
    return ARTIS_ERR_NO_CELLSTATE;
  }
  if (my_rank != G.K.R.rank) G.K.R.rank = my_rank;
  double ts = 0, tw = 0;
  // time grid lives on the device; the host copy is not kept, so read the two scalars
  HIPCHK(hipMemcpy(&ts, G.K.G.ts_start + nts, sizeof(double), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(&tw, G.K.G.ts_width + nts, sizeof(double), hipMemcpyDeviceToHost));
  const double t2 = ts + tw;
  {  // do_comp_est = do_r_lc ? false : estim_switch(nts) (sn3d.cc:539; emissivities.cc:250-257)
    DevRun &R = G.K.R;
    const double ts_want = R.time_syn_first * ((1. - G.K.G.rmax / G.K.G.tmin / ARTIS_CLIGHT_PROP));
    const double te_want = R.time_syn_last * (1. + G.K.G.rmax / G.K.G.tmin / ARTIS_CLIGHT_PROP);
    const int now = R.comp_est && !R.do_r_lc && ((ts > te_want) || (ts + tw < ts_want));
    if (now != R.comp_est_now) {
      R.comp_est_now = now;
      if (int rc = sync_ctx()) return rc;
    }
  }
  HIPCHK(hipMemsetAsync(G.K.E.err, 0, 4 * sizeof(int32_t), G.stream));
  HIPCHK(hipMemsetAsync(G.K.E.work, 0, ARTIS_WORK_COUNT * sizeof(unsigned long long), G.stream));
  const int64_t n = G.npkts;
  unsigned long long vbefore[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (G.K.V.on) {
    if (int rc = vpkt_prepare(n)) return rc;
    HIPCHK(hipMemcpy(vbefore, G.K.V.ctr, sizeof(vbefore), hipMemcpyDeviceToHost));
  }
  HIPCHK(hipEventRecord(G.ev0, G.stream));
  G.last_rounds = 0;
  if (n > 0 && G.use_megakernel) {
    if (int rc = sync_ctx()) return rc;
    k_transport<<<(unsigned)((n + TRANSPORT_BLOCK - 1) / TRANSPORT_BLOCK), TRANSPORT_BLOCK, 0, G.stream>>>(
        G.d_ctx, G.d_soa, n, nts, t2);
    HIPCHK(hipGetLastError());
    if (int rc = vpkt_flush()) return rc;
    if (G.K.V.on) {  // the megakernel does not park packets: trace the overflow records once all are done
      const DevVpkt &V = G.K.V;
      k_vpkt_ovf_copy<<<1024, 256, 0, G.stream>>>(V.ovf, V.ovf_cap, V.ovf_ctr, V.spawn, V.cap);
      k_vpkt_ovf_reset<<<1, 64, 0, G.stream>>>(V.ovf_ctr, V.ovf_cap, V.spawn_ctr, V.cap, V.full, nullptr, nullptr);
      if (int rc = vpkt_flush()) return rc;
    }
  } else if (n > 0) {
    if (int rc = run_wavefront(n, nts, t2)) return rc;
  }
  HIPCHK(hipEventRecord(G.ev1, G.stream));
  HIPCHK(hipEventSynchronize(G.ev1));
  float ms = 0.f;
  HIPCHK(hipEventElapsedTime(&ms, G.ev0, G.ev1));
  G.last_transport_ms = ms;
  if (G.K.V.on)
    if (int rc = vpkt_collect(vbefore)) return rc;
  unsigned long long w[ARTIS_WORK_COUNT];
  HIPCHK(hipMemcpy(w, G.K.E.work, sizeof(w), hipMemcpyDeviceToHost));
  for (int k = 0; k < ARTIS_WORK_COUNT; k++) G.last_work[k] = (int64_t)w[k];
  if (G.K.C.ma_level_mode && n > 0 && !G.use_megakernel) {
    // level mode: the last transport's jumps, and those made from a record (all but the wave's exact-sum jumps,
    // WaveState::stats[45])
    unsigned long long coop = 0;
    HIPCHK(hipMemcpy(&coop, G.W.stats + 45, sizeof(coop), hipMemcpyDeviceToHost));
    G.ma_acts_total = (int64_t)w[WK_MA_JUMPS];
    G.ma_acts_cached = (int64_t)w[WK_MA_JUMPS] - (int64_t)coop;
  }
  return check_kernel_error("update_packets");
}

int artis_gpu_estimators_download(artis_estimators *est) {
  if (!G.initialised) return ARTIS_ERR_NOT_INITIALISED;
  if (!est) return ARTIS_ERR_BAD_ARGUMENT;
  HIPCHK(hipStreamSynchronize(G.stream));
  const int np = G.npts_model;
  const int64_t nion_est = (int64_t)np * G.nelements * G.maxnions;
  std::vector<double> blk(G.n_est_doubles);
  HIPCHK(hipMemcpy(blk.data(), G.d_estblock, blk.size() * sizeof(double), hipMemcpyDeviceToHost));
  auto add = [&](double *dst, int64_t off, int64_t cnt) {
    if (!dst) return;
    for (int64_t j = 0; j < cnt; j++) dst[j] += blk[off + j];
  };
  add(est->J, 0, np);
  add(est->nuJ, np, np);
  add(est->ffheatingestimator, 2 * (int64_t)np, np);
  add(est->colheatingestimator, 3 * (int64_t)np, np);
  add(est->rpkt_emiss, 4 * (int64_t)np, np);
  add(est->gammaestimator, 5 * (int64_t)np, nion_est);
  add(est->bfheatingestimator, 5 * (int64_t)np + nion_est, nion_est);
  const double *sc = blk.data() + 5 * (int64_t)np + 2 * nion_est;
  est->cmf_lum += sc[0];
  est->gamma_dep += sc[1];
  est->positron_dep += sc[2];
  est->electron_dep += sc[3];
  est->electron_emission += sc[4];
  est->alpha_dep += sc[5];
  est->alpha_emission += sc[6];
  est->gamma_emission += sc[7];
  est->nt_energy_deposited += sc[8];
  est->pellet_decays += (int64_t)llrint(sc[9]);
  const int64_t off_bf = 5 * (int64_t)np + 2 * nion_est + 10;
  if (G.nbf_est) add(est->bfrate_raw, off_bf, (int64_t)np * G.nbf_est);
  if (G.nbins_est) {
    const int64_t nbn = (int64_t)np * G.nbins_est, off_rf = off_bf + (int64_t)np * G.nbf_est;
    add(est->radfield_J_raw, off_rf, nbn);
    add(est->radfield_nuJ_raw, off_rf + nbn, nbn);
    if (est->radfield_contribcount)
      for (int64_t j = 0; j < nbn; j++) est->radfield_contribcount[j] += (int64_t)llrint(blk[off_rf + 2 * nbn + j]);
  }
  if (est->compton_emiss) {  // the double sums added to the caller's float array (globals::compton_emiss)
    const int64_t off_ce = off_bf + (int64_t)np * (G.nbf_est + 3 * G.nbins_est);
    for (int64_t j = 0; j < ((int64_t)np + 1) * ARTIS_EMISS_MAX; j++)
      est->compton_emiss[j] = (float)((double)est->compton_emiss[j] + blk[off_ce + j]);
  }
  std::vector<int32_t> lc(G.nlines);
  if (est->ecounter) {
    HIPCHK(hipMemcpy(lc.data(), G.K.E.ecounter, lc.size() * sizeof(int32_t), hipMemcpyDeviceToHost));
    for (int j = 0; j < G.nlines; j++) est->ecounter[j] += lc[j];
  }
  if (est->acounter) {
    HIPCHK(hipMemcpy(lc.data(), G.K.E.acounter, lc.size() * sizeof(int32_t), hipMemcpyDeviceToHost));
    for (int j = 0; j < G.nlines; j++) est->acounter[j] += lc[j];
  }
  unsigned long long ctr[ARTIS_COUNTER_COUNT + 1];
  HIPCHK(hipMemcpy(ctr, G.K.E.counters, sizeof(ctr), hipMemcpyDeviceToHost));
  for (int j = 0; j < ARTIS_COUNTER_COUNT; j++) est->counters[j] += (int64_t)ctr[j];
  est->nesc += (int64_t)ctr[ARTIS_COUNTER_COUNT];
  return 0;
}

size_t artis_gpu_estimator_block_doubles(void) {
  if (!G.initialised) return 0;
  return (size_t)G.n_est_doubles + 2 * (size_t)G.nlines + ARTIS_COUNTER_COUNT + 1;
}

int artis_gpu_estimator_block_to_device(void *dst) {
  if (!G.initialised) return ARTIS_ERR_NOT_INITIALISED;
  double *d = (double *)dst;
  HIPCHK(hipMemcpyAsync(d, G.d_estblock, (size_t)G.n_est_doubles * sizeof(double), hipMemcpyDeviceToDevice, G.stream));
  const int64_t nc = 2 * (int64_t)G.nlines + ARTIS_COUNTER_COUNT + 1;
  k_pack_counts<<<(unsigned)((nc + 255) / 256), 256, 0, G.stream>>>(G.K.E.ecounter, G.K.E.acounter, G.K.E.counters,
                                                                     d + G.n_est_doubles, G.nlines, 0);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(G.stream));
  return 0;
}

int artis_gpu_estimator_block_from_device(const void *src) {
  if (!G.initialised) return ARTIS_ERR_NOT_INITIALISED;
  const double *s = (const double *)src;
  HIPCHK(hipMemcpyAsync(G.d_estblock, s, (size_t)G.n_est_doubles * sizeof(double), hipMemcpyDeviceToDevice, G.stream));
  const int64_t nc = 2 * (int64_t)G.nlines + ARTIS_COUNTER_COUNT + 1;
  k_pack_counts<<<(unsigned)((nc + 255) / 256), 256, 0, G.stream>>>(G.K.E.ecounter, G.K.E.acounter, G.K.E.counters,
                                                                     const_cast<double *>(s) + G.n_est_doubles,
                                                                     G.nlines, 1);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(G.stream));
  return 0;
}

// host mirror of the device block (artis_gpu_estimator_block_to_device / estimators_download)
size_t artis_estimator_block_len(int np, int ne, int mi, int nl, int nbf, int nbins) {
  if (np < 0 || ne < 0 || mi < 0 || nl < 0 || nbf < 0 || nbins < 0) return 0;
  return 5 * (size_t)np + 2 * (size_t)np * ne * mi + 10 + (size_t)np * (nbf + 3 * (size_t)nbins) +
         ((size_t)np + 1) * ARTIS_EMISS_MAX + 2 * (size_t)nl + ARTIS_COUNTER_COUNT + 1;
}

int artis_estimator_block_pack(const artis_estimators *est, int np, int ne, int mi, int nl, int nbf, int nbins,
                               double *b) {
  if (!est || !b || np < 0 || ne < 0 || mi < 0 || nl < 0 || nbf < 0 || nbins < 0) return ARTIS_ERR_BAD_ARGUMENT;
  const size_t ni = (size_t)np * ne * mi;
  auto put = [&](const double *src, size_t n) {
    for (size_t j = 0; j < n; j++) *b++ = src ? src[j] : 0.;
  };
  put(est->J, np);
  put(est->nuJ, np);
  put(est->ffheatingestimator, np);
  put(est->colheatingestimator, np);
  put(est->rpkt_emiss, np);
  put(est->gammaestimator, ni);
  put(est->bfheatingestimator, ni);
  const double sc[10] = {est->cmf_lum,        est->gamma_dep,   est->positron_dep,        est->electron_dep,
                         est->electron_emission, est->alpha_dep, est->alpha_emission,     est->gamma_emission,
                         est->nt_energy_deposited, (double)est->pellet_decays};
  put(sc, 10);
  put(est->bfrate_raw, (size_t)np * nbf);
  put(est->radfield_J_raw, (size_t)np * nbins);
  put(est->radfield_nuJ_raw, (size_t)np * nbins);
  for (size_t j = 0; j < (size_t)np * nbins; j++)
    *b++ = est->radfield_contribcount ? (double)est->radfield_contribcount[j] : 0.;
  for (size_t j = 0; j < ((size_t)np + 1) * ARTIS_EMISS_MAX; j++)
    *b++ = est->compton_emiss ? (double)est->compton_emiss[j] : 0.;
  for (int j = 0; j < nl; j++) *b++ = est->ecounter ? est->ecounter[j] : 0.;
  for (int j = 0; j < nl; j++) *b++ = est->acounter ? est->acounter[j] : 0.;
  for (int j = 0; j < ARTIS_COUNTER_COUNT; j++) *b++ = (double)est->counters[j];
  *b++ = (double)est->nesc;
  return 0;
}

int artis_estimator_block_average_scalars(double *b, int np, int ne, int mi, int nranks) {
  if (!b || np < 0 || ne < 0 || mi < 0 || nranks <= 0) return ARTIS_ERR_BAD_ARGUMENT;
  double *sc = b + 5 * (size_t)np + 2 * (size_t)np * ne * mi;
  for (int j = 0; j < 8; j++) sc[j] /= nranks;  // sn3d.cc:370-377
  return 0;
}

int artis_estimator_block_unpack(const double *b, int np, int ne, int mi, int nl, int nbf, int nbins,
                                 artis_estimators *est) {
  if (!est || !b || np < 0 || ne < 0 || mi < 0 || nl < 0 || nbf < 0 || nbins < 0) return ARTIS_ERR_BAD_ARGUMENT;
  const size_t ni = (size_t)np * ne * mi;
  auto get = [&](double *dst, size_t n) {
    if (dst)
      for (size_t j = 0; j < n; j++) dst[j] = b[j];
    b += n;
  };
  get(est->J, np);
  get(est->nuJ, np);
  get(est->ffheatingestimator, np);
  get(est->colheatingestimator, np);
  get(est->rpkt_emiss, np);
  get(est->gammaestimator, ni);
  get(est->bfheatingestimator, ni);
  est->cmf_lum = b[0];
  est->gamma_dep = b[1];
  est->positron_dep = b[2];
  est->electron_dep = b[3];
  est->electron_emission = b[4];
  est->alpha_dep = b[5];
  est->alpha_emission = b[6];
  est->gamma_emission = b[7];
  est->nt_energy_deposited = b[8];
  est->pellet_decays = (int64_t)llrint(b[9]);
  b += 10;
  get(est->bfrate_raw, (size_t)np * nbf);
  get(est->radfield_J_raw, (size_t)np * nbins);
  get(est->radfield_nuJ_raw, (size_t)np * nbins);
  for (size_t j = 0; j < (size_t)np * nbins; j++)
    if (est->radfield_contribcount) est->radfield_contribcount[j] = (int64_t)llrint(b[j]);
  b += (size_t)np * nbins;
  for (size_t j = 0; j < ((size_t)np + 1) * ARTIS_EMISS_MAX; j++)
    if (est->compton_emiss) est->compton_emiss[j] = (float)b[j];
  b += ((size_t)np + 1) * ARTIS_EMISS_MAX;
  for (int j = 0; j < nl; j++)
    if (est->ecounter) est->ecounter[j] = (int32_t)llrint(b[j]);
  b += nl;
  for (int j = 0; j < nl; j++)
    if (est->acounter) est->acounter[j] = (int32_t)llrint(b[j]);
  b += nl;
  for (int j = 0; j < ARTIS_COUNTER_COUNT; j++) est->counters[j] = (int64_t)llrint(b[j]);
  est->nesc = (int64_t)llrint(b[ARTIS_COUNTER_COUNT]);
  return 0;
}

#define NCCLCHK(x)                                                                            \
  do {                                                                                        \
    ncclResult_t r_ = (x);                                                                    \
    if (r_ != ncclSuccess) {                                                                  \
      G.last_error = std::string(#x) + ": " + ncclGetErrorString(r_);                         \
      return ARTIS_ERR_HIP;                                                                   \
    }                                                                                         \
  } while (0)

int artis_gpu_comm_unique_id(void *id) {
  if (!id) return ARTIS_ERR_BAD_ARGUMENT;
  static_assert(sizeof(ncclUniqueId) == ARTIS_COMM_ID_BYTES, "RCCL unique id size");
  ncclUniqueId uid;
  NCCLCHK(ncclGetUniqueId(&uid));
  memcpy(id, &uid, sizeof uid);
  return 0;
}

int artis_gpu_comm_init(int rank, int nranks, const void *id) {
  if (!G.initialised) return ARTIS_ERR_NOT_INITIALISED;
  if (!id || nranks <= 0 || rank < 0 || rank >= nranks) return ARTIS_ERR_BAD_ARGUMENT;
  artis_gpu_comm_finalize();
  HIPCHK(hipSetDevice(G.device));
  ncclUniqueId uid;
  memcpy(&uid, id, sizeof uid);
  NCCLCHK(ncclCommInitRank(&G.comm, nranks, uid, rank));
  G.comm_ranks = nranks;
  if (!G.d_redblock) HIPCHK(dmalloc((void **)&G.d_redblock, artis_gpu_estimator_block_doubles() * sizeof(double)));
  return 0;
}

// mpi_reduce_estimators divides the eight time_step scalars by nprocs after the sum (sn3d.cc:370-377): every rank
// carries a full-energy ensemble.  The arrays stay sums (update_grid divides them by nprocs, update_grid.cc:1041).
__global__ void k_average_timestep_scalars(double *sc, int nranks) {
  if (threadIdx.x < 8) sc[threadIdx.x] /= nranks;
}

int artis_gpu_estimators_allreduce(void) {
  if (!G.initialised) return ARTIS_ERR_NOT_INITIALISED;
  if (!G.comm || !G.d_redblock) {
    G.last_error = "artis_gpu_comm_init must precede artis_gpu_estimators_allreduce";
    return ARTIS_ERR_BAD_ARGUMENT;
  }
  if (int rc = artis_gpu_estimator_block_to_device(G.d_redblock)) return rc;
  NCCLCHK(ncclAllReduce(G.d_redblock, G.d_redblock, artis_gpu_estimator_block_doubles(), ncclFloat64, ncclSum, G.comm,
                        G.stream));
  const int64_t off_sc = 5 * (int64_t)G.npts_model + 2 * (int64_t)G.npts_model * G.nelements * G.maxnions;
  k_average_timestep_scalars<<<1, 64, 0, G.stream>>>(G.d_redblock + off_sc, G.comm_ranks);
  HIPCHK(hipGetLastError());
  return artis_gpu_estimator_block_from_device(G.d_redblock);
}

void artis_gpu_comm_finalize(void) {
  if (G.comm) {
    (void)hipStreamSynchronize(G.stream);
    (void)ncclCommDestroy(G.comm);
  }
  G.comm = nullptr;
  G.comm_ranks = 0;
}

int artis_gpu_update_packets(int my_rank, int nts, artis_packet *packets, int npkts, artis_estimators *est) {
  if (!G.initialised) return ARTIS_ERR_NOT_INITIALISED;
  if (npkts < 0 || (npkts > 0 && !packets) || !est) return ARTIS_ERR_BAD_ARGUMENT;
  int rc = artis_gpu_packets_upload(packets, npkts);
  if (rc) return rc;
  rc = artis_gpu_estimators_zero();
  if (rc) return rc;
  rc = artis_gpu_update_packets_resident(my_rank, nts);
  if (rc) return rc;
  rc = artis_gpu_packets_download(packets, npkts);
  if (rc) return rc;
  return artis_gpu_estimators_download(est);
}

}  // extern "C"
