// vpkt.h -- virtual packets (VPKT_ON, reference vpkt.cc) on the device.
//
// The reference traces, at every r-packet emission (electron scattering, macro-atom bb / fb deactivation,
// k-packet ff / fb cooling), one virtual packet per observer direction and frequency range inline, on the
// emitting packet's thread (vpkt_call_estimators vpkt.cc:837-896 -> rlc_emiss_vpkt vpkt.cc:76-368).  Here the
// emission site only records the emitting packet's state in a spawn buffer (vpkt_spawn, transport.h), and
// k_vpkt traces the virtual packets afterwards, one (spawn, observer) work item per lane:
//
//   * persistent lanes with a wave-aggregated work fetch, one cell segment (boundary, continuum opacity, the
//     lines up to the boundary, move) per loop pass, so lanes whose packet dies early (tau > tau_max) pick up
//     new work instead of idling while the wave's longest traversal runs;
//   * the per-observer cuts (time window, frequency ranges) and the order of the range loop are the
//     reference's, including the observer vector that a scattering-type traversal overwrites (vpkt.cc:179);
//   * spectra are float64 atomics into vstokes_i/q/u (add_to_vspecpol vpkt.cc:388-406) and the velocity-grid
//     map (add_to_vpkt_grid vpkt.cc:581-627).
//
// The virtual packets draw no random numbers and change nothing in the real packets, so deferring them is
// exact; only the order of the floating-point sums differs from the reference's serial loop.
#ifndef ARTIS_VPKT_H
#define ARTIS_VPKT_H

#include "wavefront.h"

#define VPKT_MAX_CELLS 1000000
// lines fetched per memory round trip in the line walk (A/B on MI355X, 1e6 packets: 4 -> 5.61 s, 8 -> 5.57 s,
// 16 -> 6.16 s)
#define VPKT_PF 8
// waves per SIMD (A/B at 1e6 packets: 1 -> 5.56 s, 2 -> 4.43 s, 3 -> 6.63 s; spills grow with the bound)
#define VPKT_OCC_DEFAULT 2

// vpkt.cc:374-385
// NS (the templates below): the spectra the loops run over, VPKT_MAX_SPECTRA or 4 when nspectra <= 4 -- the line
// walk adds each line's tau to every spectrum, and a bound of 8 cost the walk 8 masked additions per line
template <int NS = VPKT_MAX_SPECTRA>
DEVFN bool vpkt_alive(const DevVpkt &V, const double *tau) {
  int count = 0;
  for (int i = 0; i < NS; i++)
    if (i < V.nspectra && tau[i] > V.tau_max) count += 1;
  return count != V.nspectra;
}

// vpkt.cc:388-406 (deviation D9: a bin index rounded up to the array end is skipped), split in two: the time /
// frequency bin and the packet's contribution, which do not depend on the spectrum (vspec_bin, once per escaped
// virtual packet), and the three Stokes additions of one spectrum (vspec_add) -- the reference's expressions, so
// the bins and sums are add_to_vspecpol's for every spectrum
struct VspecBin {
  bool ok;
  int nt, nnu;
  double pktcontrib;
};
DEVFN VspecBin vspec_bin(const DevVpkt &V, double nu_rf, double e_rf, double t_arrive) {
  VspecBin b{false, 0, 0, 0.};
  if (t_arrive > V.tmin_vspec && t_arrive < V.tmax_vspec) {
    const int nt = (int)((log(t_arrive) - log(V.tmin_vspec)) / V.dlogt);
    if (nu_rf > V.numin_vspec && nu_rf < V.numax_vspec) {
      const int nnu = (int)((log(nu_rf) - log(V.numin_vspec)) / V.dlognu);
      if (nt >= V.vmtbins || nnu >= V.vmnubins) return b;
      b.ok = true;
      b.nt = nt;
      b.nnu = nnu;
      b.pktcontrib = e_rf / V.delta_t[nt] / V.delta_freq[nnu] / 4.e12 / ARTIS_PI / ARTIS_PARSEC / ARTIS_PARSEC /
                     V.nprocs * 4 * ARTIS_PI;
    }
  }
  return b;
}
DEVFN void vspec_add(const DevVpkt &V, const VspecBin &b, const double st[3], int bin, int ind) {
  const int ind_comb = V.nspectra * bin + ind;
  const int64_t idx = ((int64_t)b.nt * V.nobs * V.nspectra + ind_comb) * V.vmnubins + b.nnu;
#ifdef ARTIS_DIAG_NO_VSTOKES  // timing diagnostic only (drops the spectra): the cost of the escape atomics
  if (b.pktcontrib != 12345.) return;
#endif
  unsafeAtomicAdd(&V.vstokes[idx], st[0] * b.pktcontrib);
  unsafeAtomicAdd(&V.vstokes[V.vstokes_stride + idx], st[1] * b.pktcontrib);
  unsafeAtomicAdd(&V.vstokes[2 * V.vstokes_stride + idx], st[2] * b.pktcontrib);
}

// vpkt.cc:581-627
DEVFN void add_to_vpkt_grid(const Ctx &K, double nu_rf, double e_rf, const double st[3], const double vel[3],
                            int bin_range, int bin, const double obs[3]) {
  const DevVpkt &V = K.V;
  double vref1, vref2;
  const double nx = obs[0], ny = obs[1], nz = obs[2];
  if (nx == 1) {
    vref1 = vel[1];
    vref2 = vel[2];
  } else if (nx == -1) {
    vref1 = -vel[1];
    vref2 = -vel[2];
  } else {
    vref1 = -ny * vel[0] + (nx + nz * nz / (1 + nx)) * vel[1] - ny * nz * (1 - nx) / sqrt(1 - nx * nx) * vel[2];
    vref2 = -nz * vel[0] - ny * nz * (1 - nx) / sqrt(1 - nx * nx) * vel[1] + (nx + ny * ny / (1 + nx)) * vel[2];
  }
  const double vmax = K.G.vmax;
  if (fabs(vref1) >= vmax || fabs(vref2) >= vmax) return;
  const double ybin = 2 * vmax / V.ny_vgrid;
  const double zbin = 2 * vmax / V.nz_vgrid;
  const int nt = (int)((vmax - vref1) / ybin);
  const int mt = (int)((vmax - vref2) / zbin);
  if (nu_rf > V.nu_grid_min[bin_range] && nu_rf < V.nu_grid_max[bin_range]) {
    const int64_t idx = (((int64_t)nt * V.nz_vgrid + mt) * V.nrange_grid + bin_range) * V.nobs + bin;
    unsafeAtomicAdd(&V.vgrid[idx], st[0] * e_rf);
    unsafeAtomicAdd(&V.vgrid[V.vgrid_stride + idx], st[1] * e_rf);
    unsafeAtomicAdd(&V.vgrid[2 * V.vgrid_stride + idx], st[2] * e_rf);
  }
}

// state of one lane: the work item (spawn, observer, next range) and the traversal in progress
struct VLane {
  uint32_t s;
  int b, range, realtype;
  double t_current, pos0[3], obs[3];
  bool tracing;
  Pkt d;  // the dummy packet (only the fields boundary_cross / move_pkt / change_cell use are live)
  double tau[VPKT_MAX_SPECTRA];
  double I, Q, U, pn, t_future;
  int mgi, cells;
  // a line walk in progress over a coefficient row (resumed by the next pass): the segment's boundary distance and
  // next cell, the last line distance, the staged window (its lines' masks; the values are in the lane's LDS column)
  bool inlines;
  int snext, pf_base;
  double sdist, ldist;
  uint64_t wm, wm2;  // the window's line masks (lines 0-7, 8-15)
  bool esc_wait;     // escaped: waiting for the wave's next batch of escapes (k_vpkt)
#ifdef ARTIS_DIAG_VPKT_PASSES
  unsigned long long vst[5] = {0, 0, 0, 0, 0};
#endif
};

// rlc_emiss_vpkt prologue (vpkt.cc:93-193): the dummy packet, its Stokes vector and weight p_n
template <int NS>
DEVFN void vpkt_trace_init(const Ctx &K, const LocalCounters &L, VLane &v) {
  const DevVpkt &V = K.V;
  const int64_t cap = V.cap;
  const double *sp = V.spawn;
  const uint32_t s = v.s;
  const uint64_t w11 = reinterpret_cast<const uint64_t *>(sp)[11 * cap + s];
  const uint64_t w12 = reinterpret_cast<const uint64_t *>(sp)[12 * cap + s];
  Pkt &d = v.d;
  for (int k = 0; k < 3; k++) {
    d.pos[k] = v.pos0[k];
    d.dir[k] = v.obs[k];
  }
  d.where = lo32(w11);
  d.next_trans = hi32(w11);
  d.last_cross = lo32(w12);
  d.type = ARTIS_TYPE_RPKT;
  d.prop_time = v.t_current;
  d.nu_cmf = sp[6 * cap + s];
  d.e_cmf = sp[7 * cap + s];
  d.number = -1;
  for (int i = 0; i < NS; i++) v.tau[i] = 0.;
  // (nvpkt is counted by k_vpkt per lane and added once per lane at its end: a device-scope atomic on one address
  // per traced virtual packet serialised the whole kernel)
  const double t_current = v.t_current;
  const double vel_vec[3] = {v.pos0[0] / t_current, v.pos0[1] / t_current, v.pos0[2] / t_current};
  d.nu_rf = d.nu_cmf / doppler_pos_dir(K, v.pos0, d.dir, t_current);
  d.e_rf = d.e_cmf * d.nu_rf / d.nu_cmf;
  if (v.realtype == 1) {
    double Qi = sp[8 * cap + s];
    double Ui = sp[9 * cap + s];
    const double pkt_dir[3] = {sp[3 * cap + s], sp[4 * cap + s], sp[5 * cap + s]};
    double old_dir_cmf[3], obs_cmf[3], ref1[3], ref2[3];
    frame_transform(pkt_dir, &Qi, &Ui, vel_vec, old_dir_cmf);
    angle_ab(d.dir, vel_vec, obs_cmf);
    meridian(old_dir_cmf, ref1, ref2);
    const double i1 = rot_angle(old_dir_cmf, obs_cmf, ref1, ref2);
    const double cos2i1 = cos(2 * i1);
    const double sin2i1 = sin(2 * i1);
    const double Qold = Qi * cos2i1 - Ui * sin2i1;
    const double Uold = Qi * sin2i1 + Ui * cos2i1;
    const double mu = dot(old_dir_cmf, obs_cmf);
    v.pn = 3. / (16. * ARTIS_PI) * (1 + pow(mu, 2.) + (pow(mu, 2.) - 1) * Qold);
    const double Inew = 0.75 * ((mu * mu + 1.0) + Qold * (mu * mu - 1.0));
    double Qnew = 0.75 * ((mu * mu - 1.0) + Qold * (mu * mu + 1.0));
    double Unew = 1.5 * mu * Uold;
    Qnew = Qnew / Inew;
    Unew = Unew / Inew;
    v.I = Inew / Inew;
    meridian(obs_cmf, ref1, ref2);
    const double i2 = ARTIS_PI + rot_angle(obs_cmf, old_dir_cmf, ref1, ref2);
    const double cos2i2 = cos(2 * i2);
    const double sin2i2 = sin(2 * i2);
    v.Q = Qnew * cos2i2 + Unew * sin2i2;
    v.U = -Qnew * sin2i2 + Unew * cos2i2;
    const double vel_rev[3] = {-vel_vec[0], -vel_vec[1], -vel_vec[2]};
    frame_transform(obs_cmf, &v.Q, &v.U, vel_rev, v.obs);  // overwrites obs, as vpkt.cc:179
  } else {
    v.I = 1;
    v.Q = 0;
    v.U = 0;
    v.pn = 1 / (4 * ARTIS_PI);
  }
  v.mgi = cell_mgi(K, d.where);
  v.t_future = t_current;
  v.cells = 0;
  v.inlines = false;
}

// the escape branch of rlc_emiss_vpkt (vpkt.cc:314-367)
template <int NS>
DEVFN void vpkt_trace_finish(const Ctx &K, VLane &v) {
  const DevVpkt &V = K.V;
#ifdef ARTIS_DIAG_VPKT_NOFINISH  // timing diagnostic only (no spectra): the cost of the escape code
  if (v.pn != 12345.) return;
#endif
  // (nvpkt_esc1..3: counted by k_vpkt, as nvpkt)
  // t_arrive, the bins and the contribution are the same for every spectrum (computed once; the escape code runs
  // in the persistent loop's passes, where the whole wave executes it whenever one lane escapes).  Unrolled so that
  // v.tau is never indexed dynamically: one dynamic index here kept the whole lane state in scratch.
  const double t_arrive = v.t_current - (dot(v.pos0, v.d.dir) / ARTIS_CLIGHT_PROP);
  const VspecBin vb = vspec_bin(V, v.d.nu_rf, v.d.e_rf, t_arrive);
  if (vb.ok) {
#pragma unroll
    for (int ind = 0; ind < NS; ind++) {
      if (ind >= V.nspectra) break;
      const double prob = v.pn * exp(-v.tau[ind]);
      const double st[3] = {v.I * prob, v.Q * prob, v.U * prob};
      vspec_add(V, vb, st, v.b, ind);
    }
  }
  if (V.vgrid_flag == 1) {
    const double prob = v.pn * exp(-v.tau[0]);
    const double st[3] = {v.I * prob, v.Q * prob, v.U * prob};
    const double t = v.t_current;
    const double vel_vec[3] = {v.pos0[0] / t, v.pos0[1] / t, v.pos0[2] / t};
    for (int bin_range = 0; bin_range < V.nrange_grid; bin_range++)
      if (v.d.nu_rf > V.nu_grid_min[bin_range] && v.d.nu_rf < V.nu_grid_max[bin_range])
        if (t_arrive > V.tmin_grid && t_arrive < V.tmax_grid)
          add_to_vpkt_grid(K, v.d.nu_rf, v.d.e_rf, st, vel_vec, bin_range, v.b, v.obs);
  }
}

enum { VSEG_CONTINUE = 0, VSEG_ESCAPED = 1, VSEG_KILLED = 2, VSEG_PENDING = 3 };
// lines per LDS window of the walk over a coefficient row: one memory round trip per VLC_WIN lines (k_rpkt: LC_WIN).
// The phase stamps (ARTIS_DIAG_VPKT_PASSES) put 54 % of a pass in the line walk; 16-line windows (half the window
// round trips) made k_vpkt 2 % slower (3802 -> 3871 ms per 2e6-packet config-5 step, profiles/r6n_vpkt_phases.txt):
// the walk waits on its per-line dependency chain, not on the windows
#ifndef VLC_WIN
#define VLC_WIN 8
#endif
#ifndef VPKT_ESC_BATCH
#define VPKT_ESC_BATCH 16  // escaped lanes a wave gathers before running the escape code (1: at once)
#endif
#ifndef VPKT_LINE_BATCH
#define VPKT_LINE_BATCH VLC_WIN  // lines of a window evaluated side by side (1: the serial loop)
#endif
static_assert(VLC_WIN == 8 || VLC_WIN == 16, "line masks: two 64-bit words");
#ifdef ARTIS_DIAG_VPKT_PASSES  // diagnostic build: wave cycles per phase of a pass, kept by the phase's first active lane
                               // (VLane::vst) and added to g_vpkt_diag once per lane at the end
__device__ unsigned long long g_vpkt_diag[16];
#define VSTAMP_T0(t) const unsigned long long t = __builtin_amdgcn_s_memtime()
#define VSTAMP_ADD(t, slot)                                                              \
  do {                                                                                   \
    const unsigned long long _dt = __builtin_amdgcn_s_memtime() - (t);                   \
    if ((int)__lane_id() == __ffsll((long long)__ballot(1)) - 1) v.vst[(slot) - 6] += _dt;        \
  } while (0)
#else
#define VSTAMP_T0(t) \
  do {               \
  } while (0)
#define VSTAMP_ADD(t, slot) \
  do {                      \
  } while (0)
#endif
// lines a lane walks per pass of k_vpkt before the wave moves on (the walk resumes next pass): the lanes' walks
// differ in length by orders of magnitude, and an unbounded walk holds the wave for its longest lane
#ifndef VPKT_LINES_PER_PASS
#define VPKT_LINES_PER_PASS 16
#endif

// the end of a pass of rlc_emiss_vpkt's cell loop: move to the cell boundary and into the next cell (vpkt.cc:296-312)
DEVFN int vpkt_segment_end(Tx &x, VLane &v, double sdist, int snext) {
  const Ctx &K = x.K;
  Pkt &d = v.d;
  v.t_future += (sdist / ARTIS_CLIGHT_PROP);
  d.prop_time = v.t_future;
  move_pkt(K, d, sdist);
  change_cell(x, d, snext);
  const bool end_packet = (d.type == ARTIS_TYPE_ESCAPE);
  v.mgi = cell_mgi(K, d.where);
  if (v.mgi == K.G.npts_model) return VSEG_ESCAPED;
  if (K.C.thick[v.mgi] == 1) return VSEG_KILLED;
  if (++v.cells > VPKT_MAX_CELLS) {
    x.err(ERR_STUCK, -1, 6);
    return VSEG_KILLED;
  }
  return end_packet ? VSEG_ESCAPED : VSEG_CONTINUE;
}

// the line walk of a cell without a coefficient row (population gathers), whole within one pass
template <int PF, int NS>
DEVFN int vpkt_gather_walk(Tx &x, VLane &v, unsigned long long &lines, double lnu_first, double lnu_last) {
  const Ctx &K = x.K;
  const DevVpkt &V = K.V;
  Pkt &d = v.d;
  const double t_current = v.t_current;
  const double sdist = v.sdist;
  const int snext = v.snext;
  double ldist = 0;
  int pf_base = -(1 << 20);
  const double *pops = K.C.pops + (int64_t)K.C.ne_index[v.mgi] * K.T.nlevels_total;
  bool anyex = false;
  for (int ind = 0; ind < NS; ind++)
    if (ind < V.nspectra && V.exclude[ind] != 0) anyex = true;
  // As in get_event: the line records, the two populations each needs and (with element exclusions) the line's
  // atomic number are fetched PF consecutive lines at a time, all loads independent, so the walk waits for memory
  // twice per PF lines instead of three to four times per line.  The tau sums are unchanged.
  if constexpr (PF == 0) {  // launched only when every non-empty cell has a coefficient row
    x.err(ERR_UNSUPPORTED_TYPE, -1, 7);
    return VSEG_KILLED;
  } else {
  LineTau r[PF];
  double pl[PF], pu[PF];
  int z[PF] = {};
  while (ldist < sdist) {
    const int lineindex = closest_transition(K, d.nu_cmf, d.next_trans, lnu_first, lnu_last);
    if (lineindex < 0) {
      d.next_trans = K.T.nlines + 1;
      break;  // D9
    }
    if ((unsigned)(lineindex - pf_base) >= (unsigned)PF) {
      pf_base = lineindex;
      const int nl1 = K.T.nlines - 1;
#pragma unroll
      for (int q = 0; q < PF; q++) r[q] = K.T.line_tau[min(lineindex + q, nl1)];
      if (anyex) {
#pragma unroll
        for (int q = 0; q < PF; q++) z[q] = K.T.line_elem[min(lineindex + q, nl1)];
      }
#pragma unroll
      for (int q = 0; q < PF; q++) {
        pl[q] = pops[r[q].ul_lower];
        pu[q] = pops[r[q].ul_upper];
      }
    }
    const int pj = lineindex - pf_base;
    double nutrans = r[0].nu, n_u = pu[0], n_l = pl[0], B_lu = r[0].B_lu, B_ul = r[0].B_ul;
    int zl = z[0];
#pragma unroll
    for (int q = 1; q < PF; q++)
      if (pj == q) {
        nutrans = r[q].nu;
        n_u = pu[q];
        n_l = pl[q];
        B_lu = r[q].B_lu;
        B_ul = r[q].B_ul;
        zl = z[q];
      }
    d.next_trans = lineindex + 1;
    if (d.nu_cmf < nutrans)
      ldist = 0;
    else
      ldist = ARTIS_CLIGHT * t_current * (d.nu_cmf / nutrans - 1);
    if (ldist > sdist) {
      d.next_trans -= 1;
      break;
    }
    lines++;
    const double t_line = t_current + ldist / ARTIS_CLIGHT;
    const double dtau = (B_lu * n_l - B_ul * n_u) * ARTIS_HCLIGHTOVERFOURPI * t_line;
    if (!anyex) {
      for (int ind = 0; ind < NS; ind++)
        if (ind < V.nspectra) v.tau[ind] += dtau;
    } else {
      const int anumber = V.anumber[zl];
      for (int ind = 0; ind < NS; ind++)
        if (ind < V.nspectra && V.exclude[ind] != -1 && (anumber != V.exclude[ind])) v.tau[ind] += dtau;
    }
    if (!vpkt_alive<NS>(V, v.tau)) return VSEG_KILLED;
  }
  return vpkt_segment_end(x, v, sdist, snext);
  }
}

// one pass of rlc_emiss_vpkt's cell loop (vpkt.cc:195-312); deviation D9 for the line loop.  Over a coefficient
// row the line walk is resumable: it stops after VPKT_LINES_PER_PASS lines (VSEG_PENDING) and the next call continues
// it; the segment's start (boundary, continuum) runs only when no walk is in progress.
template <int PF, int NS>
DEVFN int vpkt_trace_segment(Tx &x, VLane &v, unsigned long long &lines) {
  const Ctx &K = x.K;
  const DevVpkt &V = K.V;
  Pkt &d = v.d;
  const double t_current = v.t_current;
  const double lnu_first = K.T.line_nu[0], lnu_last = K.T.line_nu[max(K.T.nlines - 1, 0)];
  const int nspec = V.nspectra;
  const double tau_max = V.tau_max;
  auto all_dead = [&]() {
    int dead = 0;
#pragma unroll
    for (int ind = 0; ind < NS; ind++)
      if (ind < nspec && v.tau[ind] > tau_max) dead++;
    return dead == nspec;
  };
  if (!v.inlines) {
    VSTAMP_T0(vt_seg);
    int snext = -1;
    const double sdist = boundary_cross(x, d, &snext);
    if (((snext != -99) && (snext < 0)) || (snext >= K.G.ngrid)) {
      x.err(ERR_BADCELL, -1, snext);
      return VSEG_KILLED;
    }
    const double tf = v.t_future;
    const double s_cont = sdist * t_current * t_current * t_current / (tf * tf * tf);
    Kappa kap;
#ifdef ARTIS_DIAG_VPKT_NOKAPPA  // timing diagnostic only (wrong opacities): the cost of the continuum evaluation
    kap.nu = d.nu_cmf;
    kap.total = kap.es = kap.ff = kap.bf = kap.ffheating = 1e-30;
#else
    calculate_kappa_rpkt_cont(x, d, K.C.ne_index[v.mgi], v.mgi, kap);
#endif
    const double kap_cont = kap.total;
    const double kap_cont_nobf = kap_cont - kap.bf;
    const double kap_cont_noff = kap_cont - kap.ff;
    const double kap_cont_noes = kap_cont - kap.es;
    for (int ind = 0; ind < NS; ind++) {
      if (ind >= V.nspectra) break;
      const double ex = V.exclude[ind];
      if (ex == -2)
        v.tau[ind] += kap_cont_nobf * s_cont;
      else if (ex == -3)
        v.tau[ind] += kap_cont_noff * s_cont;
      else if (ex == -4)
        v.tau[ind] += kap_cont_noes * s_cont;
      else
        v.tau[ind] += kap_cont * s_cont;
    }
    VSTAMP_ADD(vt_seg, 7);
    if (!vpkt_alive<NS>(V, v.tau)) return VSEG_KILLED;
    v.sdist = sdist;
    v.snext = snext;
    v.ldist = 0.;
    v.pf_base = -(1 << 20);
    v.wm = v.wm2 = 0;
    if (K.C.ne_index[v.mgi] < K.C.linecoef_rows) {
      v.inlines = true;
    } else {
      return vpkt_gather_walk<PF, NS>(x, v, lines, lnu_first, lnu_last);
    }
  }
  {
    // over the per-cell Sobolev coefficients (DevCells::linecoef, as get_event): an aligned window of LC_WIN lines'
    // frequencies and coefficients is staged in the lane's LDS column (eight independent 16-byte loads, as k_rpkt),
    // so a line reads its two values with two LDS loads instead of selecting them out of 32 registers;
    // dtau = coefficient * t_line is the reference's (B_lu n_l - B_ul n_u) * HCLIGHTOVERFOURPI * t_line in the same
    // operation order.  vpkt_alive (vpkt.cc:293) is tested when the walk leaves a window and when it ends, not after
    // every line: the tau grow with every line of positive coefficient, so a virtual packet that dies inside a window
    // is still dead there and is killed the same; a line of negative coefficient (population inversion) first checks
    // whether the packet is already dead.  Only the lines added after its death (diagnostic count) differ from the
    // reference's loop.
    const int nlines = K.T.nlines;
    const double *lnu = K.T.line_nu, *nu8 = K.T.line_nu8;
    const double *crow = K.C.linecoef + (int64_t)K.C.ne_index[v.mgi] * K.C.linecoef_stride;
    const uint8_t *lmask = V.line_mask;
    __attribute__((address_space(3))) double *win = x.win;
    const double sdist = v.sdist;
    double ldist = v.ldist;
    int pf_base = v.pf_base;
    uint64_t wm = v.wm, wm2 = v.wm2;
    int budget = VPKT_LINES_PER_PASS;
    bool done = false;
    const bool negc = __builtin_amdgcn_readfirstlane(V.neg_coef) != 0;  // (wave-uniform: a scalar branch per line)
    VSTAMP_T0(vt_walk);
#ifdef ARTIS_DIAG_VPKT_NOLINES  // timing diagnostic only (no line opacity): the cost of the line walk
    ldist = sdist;
#endif
    while (true) {
      if (!(ldist < sdist)) {
        done = true;
        break;
      }
      if (budget-- == 0) break;  // resume next pass
      const int lineindex = closest_transition(nlines, lnu, d.nu_cmf, d.next_trans, lnu_first, lnu_last);
      if (lineindex < 0) {
        d.next_trans = nlines + 1;
        done = true;
        break;  // D9
      }
      if ((unsigned)(lineindex - pf_base) >= (unsigned)VLC_WIN) {
        if (pf_base >= 0 && all_dead()) {
          v.inlines = false;
          return VSEG_KILLED;
        }
        pf_base = lineindex & ~(VLC_WIN - 1);
        lc_window_n<VLC_WIN>(nu8 + pf_base, crow + pf_base, win);
        if constexpr (VLC_WIN == 8) {
          wm = *(const __attribute__((address_space(1))) uint64_t *)(lmask + pf_base);
        } else {
          const u32x4 mw = *(glb_uint4 *)(lmask + pf_base);
          wm = mw.x | ((uint64_t)mw.y << 32);
          wm2 = mw.z | ((uint64_t)mw.w << 32);
        }
      }
#if VPKT_LINE_BATCH > 1
      // the next lines of the window as one batch: the lines are consecutive (closest_transition returns next_trans
      // once the walk is past its first line), so their distances, line times and optical depths are independent
      // and are computed side by side -- the per-line chain of two FP64 divisions was the walk's latency -- and then
      // taken in order exactly as the serial loop takes them (break at ldist > sdist, the dead-packet test at a
      // negative coefficient, the tau sums line by line)
      const int pj0 = lineindex - pf_base;
      const int nb = min(min(min(VLC_WIN - pj0, VPKT_LINE_BATCH), budget + 1), nlines - lineindex);
      budget -= nb - 1;
      const double nu_cmf = d.nu_cmf;
      double lq[VPKT_LINE_BATCH], dq[VPKT_LINE_BATCH];
#pragma unroll
      for (int q = 0; q < VPKT_LINE_BATCH; q++) {
        const int pq = min(pj0 + q, VLC_WIN - 1);
        const double nutrans = win[pq * WAVE_BLOCK_T];
        lq[q] = (nu_cmf < nutrans) ? 0. : ARTIS_CLIGHT * t_current * (nu_cmf / nutrans - 1);
        const double t_line = t_current + lq[q] / ARTIS_CLIGHT;
        dq[q] = win[(VLC_WIN + pq) * WAVE_BLOCK_T] * t_line;
      }
      bool stop = false, killed = false;
#pragma unroll
      for (int q = 0; q < VPKT_LINE_BATCH; q++) {
        if (q < nb && !stop) {
          if (q > 0 && !(ldist < sdist)) {
            done = stop = true;
          } else {
            d.next_trans = lineindex + q + 1;
            if (lq[q] > sdist) {
              ldist = lq[q];
              d.next_trans -= 1;
              done = stop = true;
            } else {
              ldist = lq[q];
              lines++;
              const int pj = pj0 + q;
              const unsigned lm = (unsigned)((pj < 8 ? wm : wm2) >> (8 * (pj & 7))) & 0xffu;
              if (negc && dq[q] < 0. && all_dead()) {
                killed = stop = true;
              } else {
#pragma unroll
                for (int ind = 0; ind < NS; ind++)
                  if ((lm >> ind) & 1u) v.tau[ind] += dq[q];
              }
            }
          }
        }
      }
      if (killed) {
        v.inlines = false;
        return VSEG_KILLED;
      }
      if (done) break;
    }
#else
      const int pj = lineindex - pf_base;
      const double nutrans = win[pj * WAVE_BLOCK_T];
      const unsigned lm = (unsigned)((pj < 8 ? wm : wm2) >> (8 * (pj & 7))) & 0xffu;
      d.next_trans = lineindex + 1;
      if (d.nu_cmf < nutrans)
        ldist = 0;
      else
        ldist = ARTIS_CLIGHT * t_current * (d.nu_cmf / nutrans - 1);
      if (ldist > sdist) {
        d.next_trans -= 1;
        done = true;
        break;
      }
      lines++;
      const double t_line = t_current + ldist / ARTIS_CLIGHT;
      const double dtau = win[(VLC_WIN + pj) * WAVE_BLOCK_T] * t_line;
      // a population inversion (NLTE) gives a negative coefficient: the only way a tau can fall again, so a
      // virtual packet that died at an earlier line of the window is killed here, before it could revive (tables
      // without a negative coefficient skip the test)
      if (negc && dtau < 0. && all_dead()) {
        v.inlines = false;
        return VSEG_KILLED;
      }
#pragma unroll
      for (int ind = 0; ind < NS; ind++)
        if ((lm >> ind) & 1u) v.tau[ind] += dtau;
    }
#endif
    VSTAMP_ADD(vt_walk, 8);
    if (!done) {
      v.ldist = ldist;
      v.pf_base = pf_base;
      v.wm = wm;
      v.wm2 = wm2;
      return VSEG_PENDING;
    }
    v.inlines = false;
    if (all_dead()) return VSEG_KILLED;
    VSTAMP_T0(vt_end);
    const int rend = vpkt_segment_end(x, v, sdist, v.snext);
    VSTAMP_ADD(vt_end, 9);
    return rend;
  }
}

// ARTIS_DIAG_VPKT_PASSES: g_vpkt_diag [0] wave passes, [1] busy lane-passes, [2] tracing lane-passes, [3] refills,
// [4] wave cycles (s_memtime), [5] cycles in refills; wave cycles in [6] the trace start (range + vpkt_trace_init),
// [7] the segment's boundary + continuum, [8] the line walk, [9] the segment's end (move, change_cell), [10] the
// escape (vpkt_trace_finish)

// all (spawn, observer) work items of the spawn buffer; spawn_ctr[1] is the fetch head
template <int PF, int MINW, int NS = VPKT_MAX_SPECTRA>
__global__ __launch_bounds__(WAVE_BLOCK, MINW) void k_vpkt(const Ctx *__restrict__ ctxp, int refill_min) {
  CTX_IN_LDS(ctxp)
  const DevVpkt &V = K.V;
  __shared__ unsigned long long s_ctr[ARTIS_COUNTER_COUNT + 1];
  __shared__ unsigned long long s_work[ARTIS_WORK_COUNT];
  block_counters_init(s_ctr, s_work);
  LocalCounters L;
  L.ctr = &s_ctr[0];
  L.work = &s_work[0];
  __shared__ double s_win[2 * VLC_WIN][WAVE_BLOCK];  // line windows of the walk over DevCells::linecoef
  static_assert(WAVE_BLOCK == WAVE_BLOCK_T, "Tx::win column stride");
  Tx x(K, L);
  x.win = (__attribute__((address_space(3))) double *)&s_win[0][threadIdx.x];
  const uint32_t nspawn = min(V.spawn_ctr[0], V.cap);
  const uint64_t nitems = (uint64_t)nspawn * (uint64_t)V.nobs;
  VLane v;
  v.tracing = false;
  v.inlines = false;
  v.esc_wait = false;
  bool have = false, drained = false;
  unsigned long long lines = 0, n_traced = 0, n_esc1 = 0, n_esc2 = 0, n_esc3 = 0;
  const int64_t cap = V.cap;
#ifdef ARTIS_DIAG_VPKT_PASSES
  unsigned long long dg[6] = {0, 0, 0, 0, 0, 0};
  const unsigned long long dg_t0 = __builtin_amdgcn_s_memtime();
#endif
  while (true) {
    const bool idle = !have && !drained;
    const unsigned long long imask = __ballot(idle);
#ifdef ARTIS_DIAG_VPKT_PASSES
    dg[0]++;
    dg[1] += __popcll(__ballot(have));
    dg[2] += __popcll(__ballot(have && v.tracing));
    const unsigned long long dg_r0 = __builtin_amdgcn_s_memtime();
#endif
    if (!__any(have) || __popcll(imask) >= refill_min) {
#ifdef ARTIS_DIAG_VPKT_PASSES
      dg[3]++;
#endif
      if (imask) {
        const uint32_t slot = wave_reserve(&V.spawn_ctr[1], idle);
        if (idle) {
          if ((uint64_t)slot < nitems) {
            if (V.perm) {
              v.b = (int)(slot / nspawn);
              v.s = V.perm[slot % nspawn];
            } else {
              v.s = slot / (uint32_t)V.nobs;
              v.b = (int)(slot % (uint32_t)V.nobs);
            }
            const double *sp = V.spawn;
            for (int k = 0; k < 3; k++) {
              v.pos0[k] = sp[k * cap + v.s];
              v.obs[k] = V.obs[3 * v.b + k];
            }
            v.t_current = sp[10 * cap + v.s];
            v.realtype = hi32(reinterpret_cast<const uint64_t *>(sp)[12 * cap + v.s]);
            const double t_arrive = v.t_current - (dot(v.pos0, v.obs) / ARTIS_CLIGHT_PROP);
            v.range = (t_arrive >= V.tmin_input && t_arrive <= V.tmax_input) ? 0 : V.nrange;
            v.tracing = false;
            have = true;
          } else {
            drained = true;
          }
        }
      }
      if (!__any(have)) break;
    }
#ifdef ARTIS_DIAG_VPKT_PASSES
    dg[5] += __builtin_amdgcn_s_memtime() - dg_r0;
#endif
    if (have && !v.esc_wait) {
      if (!v.tracing) {
        VSTAMP_T0(vt_init);
        // vpkt.cc:872-888: the next frequency range this emission falls into, with the current observer vector
        const double nu_cmf = V.spawn[6 * cap + v.s];
        while (v.range < V.nrange) {
          const double nu_rf = nu_cmf / doppler_pos_dir(K, v.pos0, v.obs, v.t_current);
          if (nu_rf > V.numin_input[v.range] && nu_rf < V.numax_input[v.range]) break;
          v.range++;
        }
        if (v.range < V.nrange) {
          v.range++;
          vpkt_trace_init<NS>(K, L, v);
          n_traced++;
          v.tracing = true;
        } else {
          have = false;
        }
        VSTAMP_ADD(vt_init, 6);
      } else {
        const int r = vpkt_trace_segment<PF, NS>(x, v, lines);
        if (r != VSEG_CONTINUE && r != VSEG_PENDING) {
          if (r == VSEG_ESCAPED) v.esc_wait = true;  // (its spectra: the wave's next batch of escapes, below)
          v.tracing = false;
        }
      }
    }
    // the escapes (spectra and velocity grid, vpkt.cc:314-367) in batches: a lane whose virtual packet escaped waits
    // until VPKT_ESC_BATCH lanes have (or no lane of the wave is tracing), so that the wave runs the escape code for
    // several lanes at once instead of for one or two in nearly every pass (11 % of a pass before, phase stamps)
    const unsigned long long em = __ballot(have && v.esc_wait);
    if (em && (__popcll(em) >= VPKT_ESC_BATCH || !__any(have && !v.esc_wait))) {
      if (have && v.esc_wait) {
        VSTAMP_T0(vt_fin);
        vpkt_trace_finish<NS>(K, v);
        VSTAMP_ADD(vt_fin, 10);
        n_esc1 += v.realtype == 1;
        n_esc2 += v.realtype == 2;
        n_esc3 += v.realtype == 3;
        v.esc_wait = false;
      }
    }
  }
#ifdef ARTIS_DIAG_VPKT_PASSES
  dg[4] = __builtin_amdgcn_s_memtime() - dg_t0;
  if (lane_id() == 0)
    for (int i = 0; i < 6; i++) atomicAdd(&g_vpkt_diag[i], dg[i]);
  for (int i = 0; i < 5; i++)
    if (v.vst[i]) atomicAdd(&g_vpkt_diag[6 + i], v.vst[i]);
#endif
  if (lines) atomicAdd(&V.ctr[6], lines);
  if (n_traced) atomicAdd(&V.ctr[0], n_traced);  // nvpkt
  if (n_esc1) atomicAdd(&V.ctr[1], n_esc1);  // nvpkt_esc1..3
  if (n_esc2) atomicAdd(&V.ctr[2], n_esc2);
  if (n_esc3) atomicAdd(&V.ctr[3], n_esc3);
  if (blockIdx.x == 0 && threadIdx.x == 0 && nspawn) atomicAdd(&V.ctr[4], (unsigned long long)nspawn);
  __syncthreads();
  if (threadIdx.x == 0) {
    if (s_work[WK_KAPPA_EVALS]) atomicAdd(&V.ctr[5], s_work[WK_KAPPA_EVALS]);
    if (s_work[WK_BF_ACTIVE]) atomicAdd(&V.ctr[7], s_work[WK_BF_ACTIVE]);
  }
  // the reference's change_cell counts virtual packets too (nesc, COUNTER_CELLCROSSINGS; boundary.cc:341-356)
  for (int j = threadIdx.x; j < ARTIS_COUNTER_COUNT + 1; j += blockDim.x)
    if (s_ctr[j]) atomicAdd(&K.E.counters[j], s_ctr[j]);
}

#endif
