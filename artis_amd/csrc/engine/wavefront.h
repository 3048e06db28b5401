// wavefront.h -- the event-queue ("wavefront") form of update_packets: one kernel per packet state.
//
// The reference advances each packet to the end of the timestep in one call chain (update_packets.cc:162-230:
// do_rpkt / do_macroatom / do_kpkt until escape or t2).  On a GPU that megakernel is a poor fit: the r-packet
// code needs ~200 live registers, so the macro-atom random walk -- most of the work, a chain of dependent
// HBM lookups -- runs at one wave per SIMD with the r-packet registers idle.  Here every state has its own
// kernel, and a packet moves between queues when its state changes:
//
//   k_rpkt : r-packet steps (rpkt.cc:1156-1283) until absorption (-> M or K queue), escape or t2
//   k_ma   : macro-atom jumps (macroatom.cc:416-482) on a 4-word lane state; never touches the packet record
//   k_kpkt : k-packet cooling (kpkt.cc:477-797) -> r-packet (R queue) or macro-atom (M queue)
//
// A macro-atom's deactivation (emission direction, fb frequency, estimator terms) is deferred to k_ma_finish,
// which loads the whole packet record (ma_finish_inl) and queues it as an r- or k-packet.  Every packet keeps its own RNG stream
// (draw counter in rng_n), so the sequence of draws -- and hence every result -- is identical to the
// megakernel and the CPU oracle.
//
// k_rpkt and k_ma are persistent: a lane that finishes its packet takes the next one from its queue
// (wave-aggregated atomic on the queue head), so lanes stay busy while walk lengths vary by orders of magnitude.
// Appends to queues are wave-aggregated (ballot + popcount + one atomic per wave).
#ifndef ARTIS_WAVEFRONT_H
#define ARTIS_WAVEFRONT_H

#include "gamma.h"

// QX: macro-atom jumps for k_ma_exact; QF: macro-atom deactivations for k_ma_finish
enum { QR = 0, QM = 1, QK = 2, QG = 3, QX = 4, QF = 5, NQUEUES = 6 };

struct WaveState {
  uint32_t *rng_n;     // [N] draws consumed so far this timestep (artis_rng.n)
  int4 *pend;          // [N] deferred macro-atom deactivation (MaEnd); .x == 0: none
  uint32_t *pend_jumps;// [N] macro-atom loop passes of that deactivation
  int32_t *q[NQUEUES]; // [N] packet indices per state
  uint32_t *ctr;       // [NQUEUES * 2]: appended count, fetch head
  // macro-atom queue binned by cell before k_ma (counting sort, order within a cell arbitrary)
  int32_t *ma_key;     // [N] nonempty-cell index of each M-queue slot
  int32_t *ma_sorted;  // [N] M queue grouped by cell (or a copy of q[QM] order when binning is off)
  uint32_t *bins;      // [n_nonempty + 1] counts, then running offsets
  uint32_t *xhead;     // [8] fetch heads of the per-XCD ranges of ma_sorted
  int ma_ranges;       // 8: blocks on XCD x take range x first (then steal), 1: one shared range
  int ma_binned;       // 1: k_ma reads ma_sorted, 0: k_ma reads q[QM]
  int bin_push;        // 1: the M queue's producers write each slot's bin (ma_key) and count it (bins) as they append
                       // it, so the binning is the scan and k_ma_scatter (no k_ma_bin pass over the queue)
  int r_binned;        // 1: this k_rpkt launch reads the R queue binned by cell from ma_sorted (k_r_bin / k_r_scatter)
  int refill_min;      // a wave refetches work (and flushes its queue appends) once this many lanes are idle
  int refill_ma;       // the same for k_ma (a macro-atom refill is cheap: one coalesced ticket read)
  int coop_max;        // level mode: at most this many cooperative jumps per k_ma pass (the other lanes without a
                       // record wait for a later pass; ARTIS_GPU_MA_COOP_MAX, default 64 = all)
  // cell-sorted macro-atom tickets written by k_ma_scatter when the key cache is on (else nullptr): per slot
  // {packet index, unique level, record offset, nonempty cell}, {packet number, RNG counter, jumps so far, 0}
  int4 *ma_tick;       // [2N]
  // the same walks' pre-tickets in M-queue order, written by the kernel that appends the walk (wave_push_ma), so
  // that the binning reads one sequential 32-byte record per slot instead of gathering the packet's words:
  // {packet index, propagation cell, packet number, RNG counter}, then {element, ion, level, 0} for a new
  // activation or {-1 - unique level, 0, 0, jumps so far} for a walk parked by k_ma_exact (nullptr: no tickets)
  int4 *ma_pre;        // [2N]
  // the F queue's records, written by the kernel that appends the deactivation (wave_push_mf): per slot
  // {MaEnd code, ion, a, b}, {jumps, RNG counter, 0, 0} -- k_ma_finish reads them with the slot, coalesced, instead of
  // gathering pend / pend_jumps / rng_n by packet index (three 64-byte sectors for 24 bytes); nullptr: those arrays
  int4 *mf_rec;        // [2N]
  unsigned long long *stats;  // [48] diagnostics: per kernel class c: [4c] wave loop passes, [4c+1] busy
                              // lane-passes, [4c+2] wave cycles (s_memtime), [4c+3] refills;
                              // [16 + 4c] cycles in refill blocks, [17 + 4c] cycles in the work step; [40] exact
                              // jumps (k_ma_exact), [45] level mode: jumps made by the wave from the exact sums
};

DEVFN int lane_id() { return (int)__lane_id(); }
// Per-pass wave diagnostics (passes, busy lanes, cycles per phase, lines scanned per pass; ARTIS_GPU_STATS=1
// prints them) are compiled in only with -DARTIS_WAVE_STATS=1 or -DARTIS_STAMPS: the s_memtime reads wait on the
// same counter as LDS traffic and the per-pass wave reductions cost LDS permutes in every pass.
#ifndef ARTIS_WAVE_STATS
#ifdef ARTIS_STAMPS
#define ARTIS_WAVE_STATS 1
#else
#define ARTIS_WAVE_STATS 0
#endif
#endif
DEVFN unsigned long long wave_clock() {
#if ARTIS_WAVE_STATS
  return __builtin_amdgcn_s_memtime();
#else
  return 0;
#endif
}
DEVFN void wave_stats_flush(const WaveState &W, int c, unsigned long long passes, unsigned long long busy,
                            unsigned long long t0, unsigned long long refills, unsigned long long trefill,
                            unsigned long long tstep) {
  if (ARTIS_WAVE_STATS && lane_id() == 0) {
    atomicAdd(&W.stats[4 * c], passes);
    atomicAdd(&W.stats[4 * c + 1], busy);
    atomicAdd(&W.stats[4 * c + 2], wave_clock() - t0);
    atomicAdd(&W.stats[4 * c + 3], refills);
    atomicAdd(&W.stats[16 + 4 * c], trefill);
    atomicAdd(&W.stats[17 + 4 * c], tstep);
  }
}

#define WAVE_BLOCK 256
#define RPKT_MAX_STEPS 2000000

// wave-aggregated reservation of one slot per lane with `pred` from counter *c; returns the lane's slot
DEVFN uint32_t wave_reserve(uint32_t *c, bool pred) {
  const unsigned long long mask = __ballot(pred);
  if (!mask) return 0xffffffffu;
  const int leader = __ffsll((long long)mask) - 1;
  uint32_t base = 0;
  if (lane_id() == leader) base = atomicAdd(c, (uint32_t)__popcll(mask));
  base = __shfl(base, leader, 64);
  const unsigned long long below = mask & ((1ull << lane_id()) - 1ull);
  return pred ? base + (uint32_t)__popcll(below) : 0xffffffffu;
}

DEVFN void wave_push(const WaveState &W, int q, bool pred, int32_t idx) {
  const uint32_t slot = wave_reserve(&W.ctr[2 * q], pred);
  if (pred) W.q[q][slot] = idx;
}
// M-queue append with the walk's pre-ticket (WaveState::ma_pre): a new macro-atom activation of packet p
// bin: the walk's M-queue bin (ma_push_bin), or -1 when the producers do not bin
DEVFN void wave_push_ma(const WaveState &W, bool pred, int32_t idx, int where, int number, uint32_t rng_n, int4 b,
                        int bin) {
  const uint32_t slot = wave_reserve(&W.ctr[2 * QM], pred);
  if (pred) {
    W.q[QM][slot] = idx;
    if (bin >= 0) {
      W.ma_key[slot] = bin;
      atomicAdd(&W.bins[bin], 1u);
    }
    if (W.ma_pre) {
      W.ma_pre[2 * (int64_t)slot] = make_int4(idx, where, number, (int)rng_n);
      W.ma_pre[2 * (int64_t)slot + 1] = b;
    }
  }
}
// F-queue append with the deactivation's record (WaveState::mf_rec)
DEVFN void wave_push_mf(const WaveState &W, bool pred, int32_t idx, int4 e, uint32_t jumps, uint32_t rng_n) {
  const uint32_t slot = wave_reserve(&W.ctr[2 * QF], pred);
  if (pred) {
    W.q[QF][slot] = idx;
    W.mf_rec[2 * (int64_t)slot] = e;
    W.mf_rec[2 * (int64_t)slot + 1] = make_int4((int)jumps, (int)rng_n, 0, 0);
  }
}
// the M-queue bin of a walk in propagation cell `where` (DevCells::ma_bin) when the producers bin
// (WaveState::bin_push), else -1
DEVFN int ma_push_bin(const Ctx &K, const WaveState &W, bool pred, int where) {
  return (W.bin_push && pred) ? K.C.ma_bin[K.C.ne_index[cell_mgi(K, where)]] : -1;
}
DEVFN int4 ma_pre_activation(int element, int ion, int level) { return make_int4(element, ion, level, 0); }
DEVFN int4 ma_pre_resume(int ul, unsigned jumps) { return make_int4(-1 - ul, 0, 0, (int)jumps); }

struct BlockCounters {
  unsigned long long *ctr, *work;
};

DEVFN void block_counters_init(unsigned long long *s_ctr, unsigned long long *s_work) {
  for (int j = threadIdx.x; j < ARTIS_COUNTER_COUNT + 1; j += blockDim.x) s_ctr[j] = 0;
  for (int j = threadIdx.x; j < ARTIS_WORK_COUNT; j += blockDim.x) s_work[j] = 0;
  __syncthreads();
}
DEVFN void block_counters_flush(const Ctx &K, const unsigned long long *s_ctr, const unsigned long long *s_work) {
  __syncthreads();
  for (int j = threadIdx.x; j < ARTIS_COUNTER_COUNT + 1; j += blockDim.x)
    if (s_ctr[j]) atomicAdd(&K.E.counters[j], s_ctr[j]);
  for (int j = threadIdx.x; j < ARTIS_WORK_COUNT; j += blockDim.x)
    if (s_work[j]) atomicAdd(&K.E.work[j], s_work[j]);
}

// update_packets.cc:280-309 prologue: reset the per-step counters of every packet, queue the active ones
__global__ void k_classify(const Ctx *__restrict__ ctxp, WaveState W, uint64_t *__restrict__ soa, int64_t n, double t2) {
  CTX_IN_LDS(ctxp)
  __shared__ unsigned long long s_ctr[ARTIS_COUNTER_COUNT + 1];
  __shared__ unsigned long long s_work[ARTIS_WORK_COUNT];
  block_counters_init(s_ctr, s_work);
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  bool toR = false, toM = false, toK = false, toG = false;
  if (i < n) {
    const uint64_t w0 = soa[PW(n, i, 0)];
    const int type = hi32(w0);
    const uint64_t w1 = soa[PW(n, i, 1)];
    soa[PW(n, i, 1)] = pack2(lo32(w1), 0);  // interactions = 0
    const uint64_t w33 = soa[PW(n, i, 33)];
    soa[PW(n, i, 33)] = pack2(0, hi32(w33));  // scat_count = 0
    const double prop_time = asd(soa[PW(n, i, 18)]);
    if (type != ARTIS_TYPE_ESCAPE && prop_time < t2) {
      atomicAdd(&s_work[WK_PACKETS_ACTIVE], 1ull);
      W.rng_n[i] = 0;
      W.pend[i] = make_int4(0, 0, 0, 0);
      toR = type == ARTIS_TYPE_RPKT;
      toM = type == ARTIS_TYPE_MA;
      toK = type == ARTIS_TYPE_KPKT || type == ARTIS_TYPE_PRE_KPKT;
      toG = is_gamma_family(type) && K.T.g_nlines;
      if (!toR && !toM && !toK && !toG) fail(K, ERR_UNSUPPORTED_TYPE, hi32(soa[PW(n, i, 33)]), type);
    }
  }
  wave_push(W, QR, toR, (int32_t)i);
  {
    int where = 0, number = 0;
    int4 b = make_int4(0, 0, 0, 0);
    if (toM) {  // (an initial macro-atom: rare)
      const uint64_t w0 = soa[PW(n, i, 0)], w36 = soa[PW(n, i, 36)], w37 = soa[PW(n, i, 37)];
      where = lo32(w0);
      number = hi32(soa[PW(n, i, 33)]);
      b = ma_pre_activation(lo32(w36), hi32(w36), lo32(w37));
    }
    wave_push_ma(W, toM, (int32_t)i, where, number, 0u, b, ma_push_bin(K, W, toM, where));
  }
  wave_push(W, QK, toK, (int32_t)i);
  wave_push(W, QG, toG, (int32_t)i);
  block_counters_flush(K, s_ctr, s_work);
}

// WALK: lines of get_event's walk a k_rpkt lane advances per pass (the walk resumes next pass); 0: whole steps
// (do_rpkt_step).  Which pays depends on the walks: on the bench (3.5 lines per step) whole steps (profiles/r4_ab.txt,
// 2e6 packets: 164 ms of k_rpkt per step, 16 lines per pass 186 ms -- the state kept across passes spills), on the
// kilonova inputs (16 lines per step, 122 for a wave's longest lane) the bounded walk (engine.hip launch_rpkt picks
// it from the previous transport's lines per step).
#ifndef RPKT_WALK_LINES
#define RPKT_WALK_LINES 16
#endif

// r-packets: persistent lanes, one r-packet step (or part of its line walk) per loop pass.  COOP: the instance for
// models with detailed bf estimators, whose continuum sums are made by the whole wave (wave_kappa_bf,
// wave_bf_estimators); the others keep the registers of the plain step.
template <int MINW, bool COOP, int WALK = 0>
__global__ __launch_bounds__(WAVE_BLOCK, MINW) void k_rpkt(const Ctx *__restrict__ ctxp, WaveState W, uint64_t *__restrict__ soa, int64_t n,
                                                     int nts, double t2) {
  CTX_IN_LDS(ctxp)
  __shared__ unsigned long long s_ctr[ARTIS_COUNTER_COUNT + 1];
  __shared__ unsigned long long s_work[ARTIS_WORK_COUNT];
  __shared__ double s_cmflum[WAVE_BLOCK / 64];
  __shared__ double s_win[2 * LC_WIN][WAVE_BLOCK];  // line windows of the walk over DevCells::linecoef
  static_assert(WAVE_BLOCK == WAVE_BLOCK_T, "Tx::win column stride");
  block_counters_init(s_ctr, s_work);
  LocalCounters L;
  L.ctr = &s_ctr[0];
  L.work = &s_work[0];
  Tx x(K, L);
  x.nts = nts;
  x.win = (__attribute__((address_space(3))) double *)&s_win[0][threadIdx.x];
  x.defer_est = true;
  // few-cell models: the block's estimator accumulator, EST_LDS_DOUBLES of dynamic LDS (none is allocated when
  // est_lds_on is false, so the other models keep k_rpkt's LDS at the line windows and the context)
  extern __shared__ double s_est[];
  const bool est_lds = est_lds_on(K);
  if (est_lds) {
    est_lds_zero(s_est);
    x.est_lds = s_est;
  }
  // models with many bf continua per frequency (detailed bf estimators: the nebular options): the step's continuum
  // sums are made by the whole wave (transport.h wave_kappa_bf / wave_bf_estimators / wave_bf_select)
  __shared__ double s_coopd[COOP ? WAVE_BLOCK * COOP_UNR : 1];
  __shared__ int s_coopi[COOP ? WAVE_BLOCK : 1];
  const bool coop = COOP && K.R.detailed_bf && K.T.nbf > 0 && K.R.do_r_lc;
  if (coop) {
    x.coop_d = &s_coopd[(threadIdx.x & ~63) * COOP_UNR];
    x.coop_i = &s_coopi[threadIdx.x & ~63];
    x.defer_bf = true;
    x.defer_sel = true;
  }
  const int npm = K.G.npts_model;
  const uint32_t nq = W.ctr[2 * QR];
  Pkt p;
  RStep S;
  bool walking = false;
  int32_t idx = -1;
  bool have = false, drained = false, pendM = false, pendK = false, pendR = false;
  int steps = 0;
  double cmf_lum = 0.;
  unsigned long long st_pass = 0, st_busy = 0, st_refill = 0, st_trefill = 0, st_tstep = 0;
  unsigned long long st_lmax = 0, st_lsum = 0, st_bmax = 0, st_bsum = 0;
  const unsigned long long st_t0 = wave_clock();
  while (true) {
    // refill only when enough lanes are idle: a refetch costs a queue atomic, the queue read and the record
    // load -- paying that on every pass for one or two finished lanes would dominate the step
    const bool idle = !have && !drained;
    const unsigned long long imask = __ballot(idle);
    if (!__any(have) || __popcll(imask) >= W.refill_min) {
      st_refill++;
      const unsigned long long tr0 = wave_clock();
      // appends deferred from the lanes' last retirement (a macro-atom: p still holds the retired packet)
      wave_push_ma(W, pendM, idx, p.where, p.number, x.rng.n, ma_pre_activation(p.ma_element, p.ma_ion, p.ma_level),
                   ma_push_bin(K, W, pendM, p.where));
      wave_push(W, QK, pendK, idx);
      wave_push(W, QR, pendR, idx);  // packets parked on a full virtual-packet buffer (resumed by the host)
      pendM = pendK = pendR = false;
      // a full virtual-packet spawn buffer: take no new packets (wave-uniform read)
      if (K.V.on && __builtin_amdgcn_readfirstlane(*(volatile uint32_t *)K.V.full)) {
        drained = true;
      } else if (imask) {
        const uint32_t slot = wave_reserve(&W.ctr[2 * QR + 1], idle);
        if (idle) {
          if (slot < nq) {
            idx = W.r_binned ? W.ma_sorted[slot] : W.q[QR][slot];
            pkt_load_hot(soa, n, idx, p);
            x.rng = artis_rng_init(K.R.seed, p.number, nts, K.R.rank);
            x.rng.n = W.rng_n[idx];
            x.ok = true;
            steps = 0;
            have = true;  // (a macro-atom deactivation was applied by k_ma_finish: no pending state here)
          } else {
            drained = true;
          }
        }
      }
      st_trefill += wave_clock() - tr0;
      if (!__any(have)) break;  // every lane is drained and its appends are flushed
    }
    st_pass++;
    st_busy += __popcll(__ballot(have));
    const unsigned long long ts0 = wave_clock();
    x.wl = x.wb = 0;
#ifdef ARTIS_STAMPS
    x.tlast = ts0;
#endif
    if (coop) {
      // the continuum opacity of the step every stepping lane is about to take (its cell and frequency at the step's
      // start, as get_event_begin evaluates it), made by the wave; unused by a step that ends before it
      bool want = false;
      int mgi = 0, k = 0;
      if (have && !x.vstop && x.ok && p.type == ARTIS_TYPE_RPKT && p.prop_time < t2) {
        mgi = cell_mgi(K, p.where);
        if (mgi != npm && K.C.thick[mgi] != 1 && K.R.opacity_case == 4) {
          want = true;
          k = K.C.ne_index[mgi];
        }
      }
      x.pre_kbf = wave_kappa_bf(x, want, k, mgi, p.nu_cmf, x.pre_hi);
      x.pre_on = want;
#ifdef ARTIS_STAMPS
      x.tlast = wave_clock();
      x.st[5] += x.tlast - ts0;
#endif
    }
    if (have) {
      // a step starts when no walk is in progress; with WALK, get_event's walk advances at most WALK lines per pass
      // (a lane with a long walk no longer holds its wave while the others' short steps wait)
      int r = -1;
      if constexpr (WALK > 0) {
        if (!walking && !x.vstop && x.ok && p.type == ARTIS_TYPE_RPKT && p.prop_time < t2) {
          r = rpkt_step_begin(x, p, t2, S);
          walking = (r == RSTEP_WALK);
        }
        if (walking && get_event_walk(x, p, S, WALK)) {
          walking = false;
          r = x.ok ? RSTEP_END : RSTEP_DONE;
        }
        if (r == RSTEP_END) rpkt_step_finish(x, p, t2, S, ColdSoa{soa, n, idx});
      } else {
        if (!x.vstop && x.ok && p.type == ARTIS_TYPE_RPKT && p.prop_time < t2) {
          do_rpkt_step(x, p, t2, ColdSoa{soa, n, idx});
          r = RSTEP_DONE;
        }
      }
      if (r == RSTEP_END || r == RSTEP_DONE) {
        STAMP(x, 4);
        if (++steps > RPKT_MAX_STEPS) x.err(ERR_STUCK, p.number, 1);
      }
    }
    // a bound-free absorption of this step: its continuum selection and the rest of the event, by the wave
    if (coop) {
#ifdef ARTIS_STAMPS
      const unsigned long long tb0 = wave_clock();
#endif
      wave_bf_select(x, p, soa, n, idx);
#ifdef ARTIS_STAMPS
      x.st[5] += wave_clock() - tb0;
#endif
    }
    if (have) {
      if (walking) {
        // (the step continues next pass)
      } else if (x.vstop && x.ok && p.type == ARTIS_TYPE_RPKT && p.prop_time < t2) {
        // its spawn went to an overflow record: park the packet (between steps) for the resumed launch
        pkt_store_hot(soa, n, idx, p);
        W.rng_n[idx] = x.rng.n;
        x.vstop = false;
        pendR = true;
        have = false;
      } else if (!x.ok || p.type != ARTIS_TYPE_RPKT || !(p.prop_time < t2)) {
        x.vstop = false;
        if (p.type == ARTIS_TYPE_ESCAPE) {
          cmf_lum += p.e_cmf;
          lwork(L, WK_ESCAPED, 1);
        }
        pkt_store_hot(soa, n, idx, p);
        // cold fields the propagation step itself writes: the escape record (change_cell, boundary.cc:332-357)
        // and the absorption record + macro-atom state of a line absorption (get_event / rpkt_event_boundbound,
        // last_event 1).  A macro-atom activated by a bf absorption (last_event 3) was set up by the cold
        // continuum-event call, which already wrote its cold words; the registers do not hold them.
        if (p.type == ARTIS_TYPE_ESCAPE) soa[PW(n, idx, 32)] = pack2(p.escape_type, p.escape_time);
        if (p.type == ARTIS_TYPE_MA && p.last_event == 1) {
#ifndef ARTIS_DIAG_NO_ABSREC  // write-traffic diagnostic only (no absorption record): its share of k_rpkt's writes
          reinterpret_cast<int32_t *>(&soa[PW(n, idx, 19)])[0] = p.absorptiontype;
          soa[PW(n, idx, 21)] = asw(p.absorptionfreq);
          for (int d = 0; d < 3; d++) soa[PW(n, idx, 22 + d)] = asw(p.absorptiondir[d]);
#endif
          soa[PW(n, idx, 36)] = pack2(p.ma_element, p.ma_ion);
          soa[PW(n, idx, 37)] = pack2(p.ma_level, p.ma_activatingline);
        } else if (p.type == ARTIS_TYPE_MA && W.ma_pre) {
          // (the continuum event set the macro-atom state on the cold copy: the pre-ticket needs it in registers)
          const uint64_t w36 = soa[PW(n, idx, 36)], w37 = soa[PW(n, idx, 37)];
          p.ma_element = lo32(w36);
          p.ma_ion = hi32(w36);
          p.ma_level = lo32(w37);
        }
        if (x.ok && p.prop_time < t2) {
          pendM = p.type == ARTIS_TYPE_MA;
          pendK = p.type == ARTIS_TYPE_KPKT || p.type == ARTIS_TYPE_PRE_KPKT;
        }
        // the RNG counter for the packet's next kernel: a macro-atom with pre-tickets carries it in its ticket
        // (wave_push_ma), and a packet that escaped or reached t2 draws nothing more this timestep
        if (pendK || (pendM && !W.ma_pre)) W.rng_n[idx] = x.rng.n;
        have = false;
      }
    }
#ifndef ARTIS_DIAG_NO_EST  // write-traffic diagnostic only (no J / nuJ / ffheating sums): their share of the writes
    wave_flush_estimators(x);  // the step's J / nuJ / ffheating terms, once per cell and wave where possible
#else
    x.est_mgi = -1;
#endif
    if (coop) {
#ifdef ARTIS_STAMPS
      const unsigned long long tb0 = wave_clock();
#endif
      wave_bf_estimators(x);
#ifdef ARTIS_STAMPS
      x.st[5] += wave_clock() - tb0;
#endif
    }
    st_tstep += wave_clock() - ts0;
    if (ARTIS_WAVE_STATS) {
      unsigned ml = x.wl, sl = x.wl, mb = x.wb, sb = x.wb;
      for (int off = 32; off > 0; off >>= 1) {
        ml = max(ml, (unsigned)__shfl_xor((int)ml, off, 64));
        sl += (unsigned)__shfl_xor((int)sl, off, 64);
        mb = max(mb, (unsigned)__shfl_xor((int)mb, off, 64));
        sb += (unsigned)__shfl_xor((int)sb, off, 64);
      }
      st_lmax += ml;
      st_lsum += sl;
      st_bmax += mb;
      st_bsum += sb;
    }
  }
#ifdef ARTIS_STAMPS
  if (lane_id() == 0)
    for (int i = 0; i < 6; i++) atomicAdd(&W.stats[32 + i], x.st[i]);
#endif
  if (ARTIS_WAVE_STATS && lane_id() == 0) {
    atomicAdd(&W.stats[24], st_lmax);
    atomicAdd(&W.stats[25], st_lsum);
    atomicAdd(&W.stats[26], st_bmax);
    atomicAdd(&W.stats[27], st_bsum);
  }
  wave_stats_flush(W, 0, st_pass, st_busy, st_t0, st_refill, st_trefill, st_tstep);
  if (est_lds) est_lds_flush(K, s_est);
  for (int off = 32; off > 0; off >>= 1) cmf_lum += __shfl_down(cmf_lum, off, 64);
  if ((threadIdx.x & 63) == 0) s_cmflum[threadIdx.x >> 6] = cmf_lum;
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0.;
    for (int w = 0; w < WAVE_BLOCK / 64; w++) s += s_cmflum[w];
    if (s != 0.) unsafeAtomicAdd(&K.E.scalars[0], s);
  }
  block_counters_flush(K, s_ctr, s_work);
}

// bin the R queue by cell before k_rpkt (the reference sorts its packets by cell before propagating them,
// update_packets.cc:204-232): lanes of a wave start in one cell, on the same linecoef row and cell state.
// Packets in empty cells share the last bin.  ma_key / ma_sorted are free while k_rpkt runs.
__global__ void k_r_bin(const Ctx *__restrict__ ctxp, WaveState W, const uint64_t *__restrict__ soa) {
  CTX_IN_LDS(ctxp)
  const uint32_t nq = W.ctr[2 * QR];
  for (uint32_t slot = blockIdx.x * blockDim.x + threadIdx.x; slot < nq; slot += gridDim.x * blockDim.x) {
    const int32_t idx = W.q[QR][slot];
    const int mgi = cell_mgi(K, lo32(soa[PW(0, idx, 0)]));  // hot group: no n term
    const int b = (mgi < K.G.npts_model) ? K.C.ne_index[mgi] : K.C.n_nonempty;
    W.ma_key[slot] = b;
    atomicAdd(&W.bins[b], 1u);
  }
}
__global__ void k_r_scatter(const Ctx *__restrict__ ctxp, WaveState W, uint32_t *offs) {
  CTX_IN_LDS(ctxp)
  const uint32_t nq = W.ctr[2 * QR];
  for (uint32_t slot = blockIdx.x * blockDim.x + threadIdx.x; slot < nq; slot += gridDim.x * blockDim.x)
    W.ma_sorted[atomicAdd(&offs[W.ma_key[slot]], 1u)] = W.q[QR][slot];
}

// the propagation cell of M-queue slot `slot`: from its pre-ticket, or the packet's hot word
DEVFN int ma_slot_where(const WaveState &W, const uint64_t *__restrict__ soa, uint32_t slot) {
  if (W.ma_pre) return W.ma_pre[2 * (int64_t)slot].y;
  return lo32(soa[PW(0, W.q[QM][slot], 0)]);  // hot group: no n term
}
// bin the M queue by cell: count per cell and remember each slot's key
__global__ void k_ma_bin(const Ctx *__restrict__ ctxp, WaveState W, const uint64_t *__restrict__ soa) {
  CTX_IN_LDS(ctxp)
  const uint32_t nq = W.ctr[2 * QM];
  for (uint32_t slot = blockIdx.x * blockDim.x + threadIdx.x; slot < nq; slot += gridDim.x * blockDim.x) {
    const int k = K.C.ne_index[cell_mgi(K, ma_slot_where(W, soa, slot))];
    const int b = K.C.ma_bin[k];
    W.ma_key[slot] = b;
    atomicAdd(&W.bins[b], 1u);
  }
}
// scatter into cell order using the exclusive prefix sum of the counts.  Each slot becomes a ticket holding
// everything k_ma's refill needs (the walk's level, record line, cell, RNG stream and jump count), so a k_ma lane
// starts a walk with one coalesced read instead of a chain of dependent packet and table loads.
// the ticket of M-queue slot `slot` at sorted position pos: from the slot's pre-ticket (WaveState::ma_pre), or
// gathered from the packet's record and side state
DEVFN void ma_ticket(const Ctx &K, const WaveState &W, const uint64_t *__restrict__ soa, int64_t n, int32_t idx,
                     uint32_t pos);
DEVFN void ma_ticket_slot(const Ctx &K, const WaveState &W, const uint64_t *__restrict__ soa, int64_t n,
                          uint32_t slot, uint32_t pos) {
  if (!W.ma_pre || !W.ma_tick) {
    ma_ticket(K, W, soa, n, W.q[QM][slot], pos);
    return;
  }
  const int4 a = W.ma_pre[2 * (int64_t)slot], b = W.ma_pre[2 * (int64_t)slot + 1];
  const int32_t idx = a.x;
  const int where = a.y, number = a.z;
  int ul;
  unsigned jumps;
  if (b.x < 0) {  // a walk parked by k_ma_exact: its level and jump count
    ul = -1 - b.x;
    jumps = (unsigned)b.w;
    W.pend[idx].x = 0;
  } else {
    ul = ulev(K, b.x, b.y, b.z);
    jumps = 0;
  }
  const int mgi = cell_mgi(K, where);
  int32_t tidx = idx;
  if (K.C.thick[mgi] == 1) {
    fail(K, ERR_THICK_MA, number, mgi);
    tidx = -1;
  }
  const int k = K.C.ne_index[mgi];
  const int32_t rowline = ma_rowline(K, k);
  W.ma_tick[2 * (int64_t)pos] = make_int4(tidx, ul, (int)ma_line(K, rowline, k, ul, K.T.ma_meta[ul].rec_off), k);
  W.ma_tick[2 * (int64_t)pos + 1] = make_int4(number, a.w, (int)jumps, rowline);
}
DEVFN void ma_ticket(const Ctx &K, const WaveState &W, const uint64_t *__restrict__ soa, int64_t n, int32_t idx,
                     uint32_t pos) {
  if (!W.ma_tick) {
    W.ma_sorted[pos] = idx;
    return;
  }
  const int where = lo32(soa[PW(n, idx, 0)]);
  const uint64_t w36 = soa[PW(n, idx, 36)], w37 = soa[PW(n, idx, 37)];
  const int number = (int)hi32(soa[PW(n, idx, 33)]);
  const int4 pd = W.pend[idx];
  int ul;
  unsigned jumps;
  if (pd.x == MA_RESUME) {  // a walk parked by k_ma_exact: continue from its level and jump count
    ul = pd.y;
    jumps = W.pend_jumps[idx];
    W.pend[idx].x = 0;
  } else {
    ul = ulev(K, lo32(w36), hi32(w36), lo32(w37));
    jumps = 0;
  }
  const int mgi = cell_mgi(K, where);
  int32_t tidx = idx;
  if (K.C.thick[mgi] == 1) {
    fail(K, ERR_THICK_MA, number, mgi);
    tidx = -1;
  }
  const int k = K.C.ne_index[mgi];
  const int32_t rowline = ma_rowline(K, k);
  W.ma_tick[2 * (int64_t)pos] = make_int4(tidx, ul, (int)ma_line(K, rowline, k, ul, K.T.ma_meta[ul].rec_off), k);
  W.ma_tick[2 * (int64_t)pos + 1] = make_int4(number, (int)W.rng_n[idx], (int)jumps, rowline);
}
__global__ void k_ma_scatter(const Ctx *__restrict__ ctxp, WaveState W, const uint64_t *__restrict__ soa, int64_t n,
                             uint32_t *offs) {
  CTX_IN_LDS(ctxp)
  const uint32_t nq = W.ctr[2 * QM];
  for (uint32_t slot = blockIdx.x * blockDim.x + threadIdx.x; slot < nq; slot += gridDim.x * blockDim.x)
    ma_ticket_slot(K, W, soa, n, slot, atomicAdd(&offs[W.ma_key[slot]], 1u));
}

// Few-cell models (n_nonempty + 1 <= MA_BIN_LDS bins: the 1D shell models, the one-zone nebular model): the same
// counting sort with block-local counts.  k_ma_bin / k_ma_scatter above add one device-scope atomic per queue entry
// to W.bins / offs; with 1, 25 or 100 bins those land on a handful of addresses and serialise (round 4: ~3.4 s of a
// 5.6 s W7-like step, ~35 s of a kilonova step).  Here each block counts a contiguous chunk of the queue in LDS and
// adds one atomic per non-empty bin; the scatter counts its chunk again, reserves the block's run of each bin with
// one atomic, and places its entries with LDS atomics.  A wave whose active lanes share one bin (the common case
// with one or few cells) adds to the LDS count once.  The order within a bin stays arbitrary (each packet draws
// from its own RNG stream: placement never changes a result).
#define MA_BIN_LDS 8192
DEVFN void ma_bin_chunk(uint32_t nq, uint32_t &lo, uint32_t &hi) {
  // contiguous chunks of whole blocks' width, at least 1024 entries: a short queue occupies few blocks
  uint32_t chunk = (nq + gridDim.x - 1) / gridDim.x;
  chunk = max(1024u, (chunk + WAVE_BLOCK - 1) / WAVE_BLOCK * WAVE_BLOCK);
  lo = min(nq, (uint32_t)blockIdx.x * chunk);
  hi = min(nq, lo + chunk);
}
// add 1 to h[b] for every active lane, return the lane's previous count (its rank); wave-uniform call
DEVFN uint32_t lds_bin_add(uint32_t *h, int b, bool active) {
  const unsigned long long am = __ballot(active);
  if (!am) return 0;
  const int lead = __ffsll((long long)am) - 1;
  const int b0 = __shfl(b, lead, 64);
  if (__all(!active || b == b0)) {
    uint32_t base = 0;
    if (lane_id() == lead) base = atomicAdd(&h[b0], (uint32_t)__popcll(am));
    base = __shfl(base, lead, 64);
    return base + (uint32_t)__popcll(am & ((1ull << lane_id()) - 1ull));
  }
  return active ? atomicAdd(&h[b], 1u) : 0u;
}
__global__ __launch_bounds__(WAVE_BLOCK) void k_ma_bin_blk(const Ctx *__restrict__ ctxp, WaveState W,
                                                           const uint64_t *__restrict__ soa) {
  CTX_IN_LDS(ctxp)
  __shared__ uint32_t h[MA_BIN_LDS];
  const uint32_t nq = W.ctr[2 * QM];
  uint32_t lo, hi;
  ma_bin_chunk(nq, lo, hi);
  if (lo >= hi) return;  // (block-uniform)
  const int nb = K.C.n_nonempty + 1;
  for (int j = threadIdx.x; j < nb; j += blockDim.x) h[j] = 0;
  __syncthreads();
  for (uint32_t s0 = lo; s0 < hi; s0 += blockDim.x) {
    const uint32_t slot = s0 + threadIdx.x;
    const bool act = slot < hi;
    int b = 0;
    if (act) {
      b = K.C.ma_bin[K.C.ne_index[cell_mgi(K, ma_slot_where(W, soa, slot))]];
      W.ma_key[slot] = b;
    }
    (void)lds_bin_add(h, b, act);
  }
  __syncthreads();
  for (int j = threadIdx.x; j < nb; j += blockDim.x)
    if (h[j]) atomicAdd(&W.bins[j], h[j]);
}
__global__ __launch_bounds__(WAVE_BLOCK) void k_ma_scatter_blk(const Ctx *__restrict__ ctxp, WaveState W,
                                                               const uint64_t *__restrict__ soa, int64_t n,
                                                               uint32_t *offs) {
  CTX_IN_LDS(ctxp)
  __shared__ uint32_t h[MA_BIN_LDS];
  const uint32_t nq = W.ctr[2 * QM];
  uint32_t lo, hi;
  ma_bin_chunk(nq, lo, hi);
  if (lo >= hi) return;
  const int nb = K.C.n_nonempty + 1;
  for (int j = threadIdx.x; j < nb; j += blockDim.x) h[j] = 0;
  __syncthreads();
  for (uint32_t s0 = lo; s0 < hi; s0 += blockDim.x) {
    const uint32_t slot = s0 + threadIdx.x;
    const bool act = slot < hi;
    (void)lds_bin_add(h, act ? W.ma_key[slot] : 0, act);
  }
  __syncthreads();
  // this block's run of every bin it holds: one device atomic per (block, bin)
  for (int j = threadIdx.x; j < nb; j += blockDim.x)
    if (h[j]) h[j] = atomicAdd(&offs[j], h[j]);
  __syncthreads();
  for (uint32_t s0 = lo; s0 < hi; s0 += blockDim.x) {
    const uint32_t slot = s0 + threadIdx.x;
    const bool act = slot < hi;
    const int key = act ? W.ma_key[slot] : 0;
    const uint32_t pos = lds_bin_add(h, key, act);
    if (act) ma_ticket_slot(K, W, soa, n, slot, pos);
  }
}

// macro-atoms: persistent lanes, one jump per loop pass, lane state = MaLaneR + RNG counter.
// The (binned) queue is cut into W.ma_ranges contiguous ranges; blocks start on range blockIdx % 8 -- the
// XCD the block was dispatched to under round-robin placement, so one XCD's L2 sees a contiguous run of
// cells -- and steal from the following ranges once theirs is exhausted.
// A lane whose (cell, level) has a key record takes the cached step (ma_step_cached, its record line staged in
// LDS by the wave's cooperative fetch); a lane without one (level mode, DevCells::ma_lptr) has its jump made by
// the whole wave after the cached steps (ma_coop_select), one such lane after another.
// COOP = false (row mode: every pair has a record) compiles without the cooperative jump.
// LEVEL (level mode, DevCells::ma_lptr): a lane without a record -- or whose high key halves cannot decide -- makes
// that jump in the wave's exact-sum path: inline in this pass (COOP), or parked on the QX queue for k_ma_exact.
template <int MINW, bool COOP, bool LEVEL>
__global__ __launch_bounds__(WAVE_BLOCK, MINW) void k_ma(const Ctx *__restrict__ ctxp, WaveState W,
                                                         const uint64_t *__restrict__ soa, int64_t n, int nts) {
  CTX_IN_LDS(ctxp)
  __shared__ unsigned long long s_ctr[ARTIS_COUNTER_COUNT + 1];
  __shared__ unsigned long long s_work[ARTIS_WORK_COUNT];
  // per wave: the 128-byte hot line of each lane's current macro-atom record (ma_jump_cached), chunk-major
  __shared__ uint4 s_line[WAVE_BLOCK / 64][8 * 64];
  __shared__ __attribute__((aligned(16))) uint64_t s_xidx[WAVE_BLOCK / 64][64];  // line addresses exchanged for the cooperative fetch
  block_counters_init(s_ctr, s_work);
  LocalCounters L;
  L.ctr = &s_ctr[0];
  L.work = &s_work[0];
  lds_uint4 *line = (lds_uint4 *)&s_line[threadIdx.x >> 6][threadIdx.x & 63];
  const uint32_t nq = W.ctr[2 * QM];
  const int32_t *queue = W.ma_binned ? W.ma_sorted : W.q[QM];
  const int nr = W.ma_ranges;
  const int nr_log2 = (nr == 8) ? 3 : 0;  // W.ma_ranges is 1 or 8
  const double t_mid = K.G.ts_mid[nts];
  [[maybe_unused]] const int lane = lane_id();
  const MaHot H = ma_hot(*ctxp);  // (scalar loads from the device context: kept in SGPRs, MaHot)
  MaLaneR mc;
  artis_rng rng = artis_rng_init(K.R.seed, 0, nts, K.R.rank);
  int32_t idx = -1;
  bool have = false, drained = false;
  int cur = (int)(blockIdx.x % (unsigned)nr), tried = 0;
  bool pendF = false, pendX = false;
  int4 fe = make_int4(0, 0, 0, 0);  // a deactivation waiting for the F-queue append: its record (WaveState::mf_rec)
  uint32_t fjumps = 0, frng = 0;
  unsigned long long jumps_sum = 0, trans_sum = 0, coop_sum = 0;
  unsigned long long st_pass = 0, st_busy = 0, st_refill = 0, st_trefill = 0, st_tstep = 0;
#ifdef ARTIS_STAMPS
  unsigned long long ma_st[4] = {0, 0, 0, 0};
  __shared__ unsigned long long s_diag[48];
  for (int j = threadIdx.x; j < 48; j += blockDim.x) s_diag[j] = 0;
  __syncthreads();
  L.diag = s_diag;
#endif
  const unsigned long long st_t0 = wave_clock();
  int refill_ma = W.refill_ma;
  asm volatile("" : "+s"(refill_ma));  // (held in an SGPR: not reloaded from the kernel arguments every pass)
  while (true) {
    const bool idle = !have && !drained;
    const unsigned long long imask = __ballot(idle);
    if (!__any(have) || __popcll(imask) >= refill_ma) {
      st_refill++;
      const unsigned long long tr0 = wave_clock();
      if (W.mf_rec)
        wave_push_mf(W, pendF, idx, fe, fjumps, frng);
      else
        wave_push(W, QF, pendF, idx);
      wave_push(W, QX, pendX, idx);
      pendF = pendX = false;
      if (imask) {
        // (nr is 1 or 8: shifts, not the 64-bit division the compiler would expand into ~120 scalar instructions)
        const uint32_t lo = (uint32_t)(((uint64_t)nq * cur) >> nr_log2),
                       hi = (uint32_t)(((uint64_t)nq * (cur + 1)) >> nr_log2);
        const uint32_t slot = wave_reserve(&W.xhead[cur], idle);
        const bool got = idle && lo + slot < hi;
        if (got && W.ma_tick) {
          const int4 t0 = W.ma_tick[2 * (int64_t)(lo + slot)], t1 = W.ma_tick[2 * (int64_t)(lo + slot) + 1];
          idx = t0.x;
          mc.ul = t0.y;
          mc.line = (uint32_t)t0.z;
          mc.k = t0.w;
          rng.key1 = (uint32_t)t1.x;
          rng.n = (uint32_t)t1.y;
          mc.jumps = (unsigned)t1.z;
          mc.rowline = t1.w;
          mc.ntrans = 0;
          mc.sel = -1;
          mc.pline = 0;
          have = idx >= 0;
        } else if (got) {
          idx = queue[lo + slot];
          const int where = lo32(soa[PW(n, idx, 0)]);
          const uint64_t w36 = soa[PW(n, idx, 36)];
          const uint64_t w37 = soa[PW(n, idx, 37)];
          rng.key1 = (uint32_t)hi32(soa[PW(n, idx, 33)]);  // packet number
          rng.n = W.rng_n[idx];
          const int mgi = cell_mgi(K, where);
          const int4 pd = W.pend[idx];
          mc.k = K.C.ne_index[mgi];
          mc.rowline = ma_rowline(K, mc.k);
          if (pd.x == MA_RESUME) {  // a walk parked by k_ma_exact: continue from its level and jump count
            ma_set_level(H, mc, pd.y);
            mc.jumps = W.pend_jumps[idx];
            W.pend[idx].x = 0;
          } else {
            ma_set_level(H, mc, ulev(K, lo32(w36), hi32(w36), lo32(w37)));
            mc.jumps = 0;
          }
          mc.ntrans = 0;
          mc.sel = -1;
          mc.pline = 0;
          have = true;
          if (K.C.thick[mgi] == 1) {
            fail(K, ERR_THICK_MA, (int)rng.key1, mgi);
            have = false;
          }
        }
        if (__any(idle && !got)) {  // this range is used up: move on (wave-uniform)
          cur = (cur + 1) % nr;
          if (++tried >= nr) drained = true;
        }
      }
      st_trefill += wave_clock() - tr0;
      if (!__any(have)) {
        if (drained) break;
        continue;
      }
    }
    st_pass++;
    st_busy += __popcll(__ballot(have));
    const unsigned long long ts0 = wave_clock();
    // a lane whose current level has no record: its jump is made by the whole wave below
    const bool unc = LEVEL && have && mc.line == MA_NOLINE;
    MaMetaW meta;
    u32x4 zw = {0u, 0u, 0u, 0u};
    {
      // the level's metadata and, 8 lines per load instruction, every busy lane's record line; the lane's next two
      // draws are computed while they are in flight
      if (have) meta = ma_walk_load(H.ma_walk, mc.ul);
      const uint32_t myline = (have && !unc) ? mc.line + (uint32_t)mc.pline : 0u;  // (idle lanes: a harmless line 0)
      WaveLines wl;
      wave_fetch_issue(H.ma_key, myline, wl, (lds_u64 *)&s_xidx[threadIdx.x >> 6][0]);
      if (have && mc.sel < 0) {
#ifdef ARTIS_DIAG_CHEAPRNG  // timing diagnostic only (wrong stream): the walk's cost without Philox
        uint64_t h = ((uint64_t)rng.key1 << 32) ^ rng.n;
        h = (h ^ (h >> 30)) * 0xbf58476d1ce4e5b9ull;
        zw = u32x4{(uint32_t)h, (uint32_t)(h >> 32), (uint32_t)(h >> 16), (uint32_t)(h >> 40)};
#else
        // (the jump's two draws, one Philox block, kept as words: include/artis_rng.h, ma_qh_draw)
        artis_rng_jump_words(&rng, (uint32_t *)&zw);
#endif
      }
      wave_fetch_commit(wl, line - (threadIdx.x & 63));
    }
#ifdef ARTIS_STAMPS
    const unsigned long long ts1 = wave_clock();
    unsigned long long ts2 = ts1;
#endif
    MaEnd e;
    int r = MA_PENDING;
    if (have && !unc) {
      r = ma_step_cached(K, H, L, rng, mc, e, (int)rng.key1, KeysLds<LEVEL && ARTIS_MA_HI_ONLY>{line, mc.pline}, meta,
                         zw);
#ifdef ARTIS_STAMPS
      ts2 = wave_clock();
#endif
    }
    // level mode: a jump the high key halves cannot decide is made by the wave below from the exact sums, with the
    // lane's RNG counter back at the start of the jump (the same draws), not parked for k_ma_exact
    if (LEVEL && !COOP && unc) {  // -> k_ma_exact (a jump not yet begun: its draws start at the current counter)
      mc.n0 = rng.n;
      r = MA_DEFER;
    }
    bool unc_now = unc;
    if (COOP && r == MA_DEFER) {
      rng.n = mc.n0;
      // (a search that began in an earlier pass has no draws computed in this one)
      artis_rng_jump_words(&rng, (uint32_t *)&zw);
      unc_now = true;
      r = MA_PENDING;
    }
    // level mode: the jumps of the lanes without a record, each made by the whole wave (wave-uniform loop)
    if constexpr (COOP) {
      // the action of every such lane from its pair's totals, lane by lane; a collisional / NT action (or the
      // abort) is applied at once, a transition action waits for the wave's search of its list
      int csel = MA_COOP_RANDOM;
      double cx = 0.;
      if (unc_now) {
        csel = ma_coop_action(K, mc.k, mc.ul, artis_rng_word_unit(zw.x, zw.y), artis_rng_word_unit(zw.z, zw.w), &cx);
        if (!ma_coop_needs_search(csel)) {
          r = ma_coop_apply(K, H, L, rng, mc, e, (int)rng.key1, csel, -1, 0u, meta);
          coop_sum++;
        }
      }
      // (a rotating start, so that with coop_max < 64 every waiting lane gets its turn)
      unsigned long long um = __ballot(unc_now && ma_coop_needs_search(csel));
      const int rot = (int)(st_pass & 63);
      um = (um >> rot) | (rot ? um << (64 - rot) : 0ull);
      for (int done_coop = 0; um && done_coop < W.coop_max; um &= um - 1, done_coop++) {
        const int ld = (__ffsll((long long)um) - 1 + rot) & 63;
        const int ul = __builtin_amdgcn_readlane(mc.ul, ld), k = __builtin_amdgcn_readlane(mc.k, ld);
        const int sl = __builtin_amdgcn_readlane(csel, ld);
        int j = -1;
        unsigned probes = 0;
        const int sel = ma_coop_search(K, k, ul, sl, readlane_d(cx, ld), t_mid, &j, probes);
        if (lane == ld) {
          r = ma_coop_apply(K, H, L, rng, mc, e, (int)rng.key1, sel, j, probes, meta);
          coop_sum++;
        }
      }
    }
    if (have) {
      const unsigned jumps = mc.jumps;
      if (r == MA_DEFER) {  // park the walk before this jump; k_ma_exact makes it with the exact sums
        W.pend[idx] = make_int4(MA_RESUME, mc.ul, 0, 0);
        W.pend_jumps[idx] = jumps;
        W.rng_n[idx] = mc.n0;
        trans_sum += mc.ntrans;
        pendX = true;
        have = false;
      }
      if (have && r != MA_PENDING && (r != MA_CONTINUE || jumps >= MA_MAX_JUMPS)) {
        if (r == MA_CONTINUE) fail(K, ERR_STUCK, (int)rng.key1, 2);
        if (r > 0) {
          if (W.mf_rec) {
            fe = make_int4(e.code, e.ion, e.a, e.b);
            fjumps = jumps;
            frng = rng.n;
          } else {
            W.pend[idx] = make_int4(e.code, e.ion, e.a, e.b);
            W.pend_jumps[idx] = jumps;
            W.rng_n[idx] = rng.n;
          }
          pendF = true;  // -> k_ma_finish
        }
        jumps_sum += jumps;
        trans_sum += mc.ntrans;
        have = false;
      }
    }
    st_tstep += wave_clock() - ts0;
#ifdef ARTIS_STAMPS
    // k_ma phases (cycles per pass): fetch (metadata + record lines in LDS), jump, the rest of the pass; with
    // ARTIS_STAMPS_TWAIT the pass first waits for every outstanding load (the transition-target loads) and that
    // wait is its own phase
    {
      unsigned long long t2max = ts2;
      for (int off = 32; off > 0; off >>= 1) t2max = max(t2max, (unsigned long long)__shfl_xor((long long)t2max, off, 64));
      ma_st[0] += ts1 - ts0;
      ma_st[1] += t2max - ts1;
#ifdef ARTIS_STAMPS_TWAIT
      __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
      const unsigned long long tw = wave_clock();
      ma_st[3] += tw - t2max;
      t2max = tw;
#endif
      ma_st[2] += wave_clock() - t2max;
    }
#endif
  }
#ifdef ARTIS_STAMPS
  if (lane_id() == 0)
    for (int i = 0; i < 3; i++) atomicAdd(&W.stats[41 + i], ma_st[i]);
  if (lane_id() == 0) atomicAdd(&W.stats[44], ma_st[3]);
  __syncthreads();
  for (int j = threadIdx.x; j < 48; j += blockDim.x)
    if (s_diag[j]) atomicAdd(&g_ma_diag[j], s_diag[j]);
#endif
  wave_stats_flush(W, 1, st_pass, st_busy, st_t0, st_refill, st_trefill, st_tstep);
  if (jumps_sum) atomicAdd(&s_work[WK_MA_JUMPS], jumps_sum);
  if (coop_sum) atomicAdd(&W.stats[45], coop_sum);  // (level mode: jumps made by the wave from the exact sums)
  if (trans_sum) atomicAdd(&s_work[WK_MA_TRANS], trans_sum);
  block_counters_flush(K, s_ctr, s_work);
}

// macro-atom jumps whose key comparisons were undecided (QX): one jump each with the reference's exact sums, then
// the walk is parked again for k_ma (-> M queue) or its deactivation deferred like k_ma's (-> R / K queue).
// One wave per jump: the lanes evaluate the level's individual rates (ma_rate_at, the expressions of
// ma_foreach_rate) MAXCH at a time into LDS, and every lane then sums them in the reference's order
// (macroatom.cc:57-159, 502-525) -- the same sums as the single-thread ma_jump_exact, without its chain of
// dependent loads.  Rare (~1 per 10^5 jumps), so blocks of one wave, grid-stride over the queue.
#define MAX_CH 256
__global__ __launch_bounds__(64) void k_ma_exact(const Ctx *__restrict__ ctxp, WaveState W,
                                                 const uint64_t *__restrict__ soa, int64_t n, int nts) {
  CTX_IN_LDS(ctxp)
  __shared__ unsigned long long s_ctr[ARTIS_COUNTER_COUNT + 1];
  __shared__ unsigned long long s_work[ARTIS_WORK_COUNT];
  __shared__ double s_R[MAX_CH], s_C[MAX_CH], s_et[MAX_CH], s_eg[MAX_CH];
  __shared__ int s_kind[MAX_CH], s_j[MAX_CH];
  block_counters_init(s_ctr, s_work);
  LocalCounters L;
  L.ctr = &s_ctr[0];
  L.work = &s_work[0];
  const int lane = threadIdx.x & 63;
  const uint32_t nq = W.ctr[2 * QX];
  const double t_mid = K.G.ts_mid[nts];
  unsigned long long n_exact = 0;  // exact jumps of this block (lane 0)
  // the walks' next queue, gathered over the wave's lanes (lane j holds the j-th pending append) and appended 64 at a
  // time: one queue atomic per 64 jumps instead of one per jump on the queue's counter
  int32_t pm = -1, pf = -1;
  int nm = 0, nf = 0;
  int4 pf_e = make_int4(0, 0, 0, 0);  // the pending F appends' records (WaveState::mf_rec)
  uint32_t pf_jumps = 0, pf_rng = 0;
  int pm_where = 0, pm_number = 0, pm_ul = 0;  // the pending M appends' pre-tickets (WaveState::ma_pre)
  uint32_t pm_rng = 0, pm_jumps = 0;
  auto flush = [&](bool all) {
    if (all || nm == 64) {
      wave_push_ma(W, lane < nm, pm, pm_where, pm_number, pm_rng, ma_pre_resume(pm_ul, pm_jumps),
                   ma_push_bin(K, W, lane < nm, pm_where));
      nm = 0;
    }
    if (all || nf == 64) {
      if (W.mf_rec)
        wave_push_mf(W, lane < nf, pf, pf_e, pf_jumps, pf_rng);
      else
        wave_push(W, QF, lane < nf, pf);
      nf = 0;
    }
  };
  // lane 0's decision for this slot; a walk parked again: its level, jump count and RNG counter (lane 0's) and
  // cell / packet number (wave-uniform)
  auto collect = [&](int32_t to_m, int32_t to_f, int where, int number, int ul, unsigned jumps, uint32_t rngn,
                     int4 fe) {
    const int32_t m = __builtin_amdgcn_readlane(to_m, 0), f = __builtin_amdgcn_readlane(to_f, 0);
    const int ul0 = __builtin_amdgcn_readlane(ul, 0);
    const uint32_t j0 = (uint32_t)__builtin_amdgcn_readlane((int)jumps, 0), r0 = (uint32_t)__builtin_amdgcn_readlane((int)rngn, 0);
    if (m >= 0) {
      if (lane == nm) {
        pm = m;
        pm_where = where;
        pm_number = number;
        pm_ul = ul0;
        pm_jumps = j0;
        pm_rng = r0;
      }
      nm++;
    }
    if (f >= 0) {
      const int4 e0 = make_int4(__builtin_amdgcn_readlane(fe.x, 0), __builtin_amdgcn_readlane(fe.y, 0),
                                __builtin_amdgcn_readlane(fe.z, 0), __builtin_amdgcn_readlane(fe.w, 0));
      if (lane == nf) {
        pf = f;
        pf_e = e0;
        pf_jumps = j0;
        pf_rng = r0;
      }
      nf++;
    }
    flush(false);
  };
  for (uint32_t slot = blockIdx.x; slot < nq; slot += gridDim.x) {
    const int32_t idx = W.q[QX][slot];
    int32_t to_m = -1, to_f = -1;  // (set by lane 0)
    const int where = lo32(soa[PW(n, idx, 0)]);
    artis_rng rng = artis_rng_init(K.R.seed, (int)hi32(soa[PW(n, idx, 33)]), nts, K.R.rank);
    rng.n = W.rng_n[idx];
    const int number = (int)rng.key1;
    MaLaneC m;
    m.ul = W.pend[idx].y;
    m.jumps = W.pend_jumps[idx] + 1;
    m.k = K.C.ne_index[cell_mgi(K, where)];
    m.rowline = ma_rowline(K, m.k);
    m.line = MA_NOLINE;  // (the walk resumes in k_ma, whose ticket looks its record up again)
    m.ntrans = 0;
    const int ul = m.ul, k = m.k;
    if (K.C.ma_level_mode) {
      // level mode (a pair without a record, or a comparison its high key halves could not decide): the action from
      // the pair's exact totals, the transition by the wave's search -- k_ma's exact-sum jump (ma_coop_action /
      // ma_coop_search / ma_coop_apply), the same draws and sums
      double z1, z2;
      artis_rng_jump_pair(&rng, &z1, &z2);
      double x = 0.;
      int sel = ma_coop_action(K, k, ul, z1, z2, &x);
      int j = -1;
      unsigned probes = 0;
      if (ma_coop_needs_search(sel)) sel = ma_coop_search(K, k, ul, sel, x, t_mid, &j, probes);
      int res_ul = 0;
      unsigned res_jumps = 0;
      int4 res_e = make_int4(0, 0, 0, 0);
      if (lane == 0) {
        MaLaneR mr;
        static_cast<MaLaneC &>(mr) = m;
        mr.jumps = W.pend_jumps[idx];  // (ma_coop_apply counts the jump)
        MaEnd e{};
        const int r = ma_coop_apply(K, ma_hot(K), L, rng, mr, e, number, sel, j, probes, ma_walk_load(K, ul));
        lwork(L, WK_MA_TRANS, mr.ntrans);
        n_exact++;  // (stats[40], [45]: added once per block, not once per jump on one address)
        W.rng_n[idx] = rng.n;
        W.pend_jumps[idx] = mr.jumps;
        if (r == MA_CONTINUE) {
          if (mr.jumps >= MA_MAX_JUMPS) {
            fail(K, ERR_STUCK, number, 2);
          } else {
            W.pend[idx] = make_int4(MA_RESUME, mr.ul, 0, 0);
            to_m = idx;
          }
        } else if (r > 0) {
          res_e = make_int4(e.code, e.ion, e.a, e.b);
          if (!W.mf_rec) W.pend[idx] = res_e;
          lwork(L, WK_MA_JUMPS, mr.jumps);
          to_f = idx;  // -> k_ma_finish
        }
        res_ul = mr.ul;
        res_jumps = mr.jumps;
      }
      collect(to_m, to_f, where, number, res_ul, res_jumps, rng.n, res_e);
      continue;
    }
    const int mgi = K.C.ne_mgi[k];
    const MaMeta mm = K.T.ma_meta[ul];
    const int cnt = mm.nd + mm.nr + mm.nu + mm.nt;
    const double ec = K.T.level_epsilon[ul];
    const double *pops = K.C.pops + (int64_t)k * K.T.nlevels_total;
    const double *corr = K.C.corrphot + (int64_t)k * K.T.ntargets_total;
    auto pop = [&](int u) { return pops[u]; };
    auto cph = [&](int s) { return corr[s]; };
    // rates of positions [c0, c0 + MAX_CH) into LDS, one per lane per pass
    auto fill = [&](int c0) {
      __syncthreads();
      for (int q = lane; q < MAX_CH && c0 + q < cnt; q += 64) {
        const MaItem it = ma_rate_at(K, mgi, ul, t_mid, c0 + q, pop, cph);
        s_R[q] = it.R;
        s_C[q] = it.C;
        s_et[q] = it.et;
        s_eg[q] = it.eg;
        s_kind[q] = it.kind;
        s_j[q] = it.j;
      }
      __syncthreads();
    };
    double pr[ARTIS_MA_ACTION_COUNT];
    for (int a = 0; a < ARTIS_MA_ACTION_COUNT; a++) pr[a] = 0.;
    for (int c0 = 0; c0 < cnt; c0 += MAX_CH) {
      fill(c0);
      for (int q = 0; q < MAX_CH && c0 + q < cnt; q++) ma_accumulate(pr, s_kind[q], s_R[q], s_C[q], s_et[q], s_eg[q], ec);
    }
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
    MaEnd e{};
    int r;
    if (rate <= randomrate) {
      if (lane == 0) fail(K, ERR_MA_RANDOM, number, ul);
      r = MA_FAILED;
    } else if (sel == ARTIS_MA_ACTION_COLDEEXC || sel == ARTIS_MA_ACTION_COLRECOMB) {
      e.code = (sel == ARTIS_MA_ACTION_COLDEEXC) ? MA_END_COLDEEXC : MA_END_COLRECOMB;
      r = e.code;
    } else if (sel == ARTIS_MA_ACTION_INTERNALUPHIGHERNT) {
      r = (lane == 0) ? ma_apply_nt(K, L, rng, m, number) : MA_CONTINUE;
    } else {
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
      for (int c0 = 0; c0 < cnt && found < 0; c0 += MAX_CH) {
        fill(c0);
        for (int q = 0; q < MAX_CH && c0 + q < cnt; q++) {
          ma_accumulate(run, s_kind[q], s_R[q], s_C[q], s_et[q], s_eg[q], ec);
          if (s_kind[q] == kind) m.ntrans++;
          if (s_kind[q] == kind && run[sel] > x) {
            found = s_j[q];
            break;
          }
        }
      }
      if (found < 0) {
        if (lane == 0) fail(K, ERR_MA_SELECT, number, 10 + sel);
        r = MA_FAILED;
      } else {
        r = (lane == 0) ? ma_apply_selection(K, ma_hot(K), L, m, e, sel, found, mm.doff, mm.uoff, mm.base_lower)
                        : MA_CONTINUE;
      }
    }
    if (lane == 0) {
      lwork(L, WK_MA_TRANS, m.ntrans);
      n_exact++;
      W.rng_n[idx] = rng.n;
      W.pend_jumps[idx] = m.jumps;
      if (r == MA_CONTINUE) {
        if (m.jumps >= MA_MAX_JUMPS) {
          fail(K, ERR_STUCK, number, 2);
        } else {
          W.pend[idx] = make_int4(MA_RESUME, m.ul, 0, 0);
          to_m = idx;
        }
      } else if (r > 0) {
        if (!W.mf_rec) W.pend[idx] = make_int4(e.code, e.ion, e.a, e.b);
        lwork(L, WK_MA_JUMPS, m.jumps);
        to_f = idx;  // -> k_ma_finish
      }
    }
    collect(to_m, to_f, where, number, m.ul, m.jumps, rng.n, make_int4(e.code, e.ion, e.a, e.b));
  }
  flush(true);
  if (lane == 0 && n_exact) {
    atomicAdd(&W.stats[40], n_exact);                    // diagnostics: exact jumps
    if (K.C.ma_level_mode) atomicAdd(&W.stats[45], n_exact);  // level mode: jumps made from the exact sums
  }
  block_counters_flush(K, s_ctr, s_work);
}

// macro-atom deactivations (the F queue, filled by k_ma and k_ma_exact): the deactivation branches of do_macroatom
// (macroatom.cc:222-380) and its trailer (macroatom.cc:475-482) on the whole packet in registers, one packet per
// lane, then -> R (bb / fb emission) or K (collisional deactivation).  Until round 4 k_rpkt / k_kpkt applied the
// deactivation when they picked the packet up, as a noinline call on a scratch copy of the packet: in k_rpkt that
// copy (~400 B per lane written and read back once per macro-atom cycle) was most of the kernel's write traffic.
// With virtual packets the slots are taken from the fetch head and a full spawn buffer stops the launch (each lane
// spawns at most once, so the overflow records cover the lanes in flight), as in k_kpkt.
#ifndef MA_FINISH_MINW
#define MA_FINISH_MINW 1  // waves per SIMD k_ma_finish is compiled for
#endif
__global__ __launch_bounds__(WAVE_BLOCK, MA_FINISH_MINW) void k_ma_finish(const Ctx *__restrict__ ctxp, WaveState W,
                                                          uint64_t *__restrict__ soa, int64_t n, int nts, double t2) {
  CTX_IN_LDS(ctxp)
  __shared__ unsigned long long s_ctr[ARTIS_COUNTER_COUNT + 1];
  __shared__ unsigned long long s_work[ARTIS_WORK_COUNT];
  __shared__ double s_fbP[WAVE_BLOCK / 64][WAVE_FB_MAXP + 1];  // the waves' fb running sums (wave_select_continuum_nu)
  lds_double *fbP = (lds_double *)&s_fbP[threadIdx.x >> 6][0];
  block_counters_init(s_ctr, s_work);
  LocalCounters L;
  L.ctr = &s_ctr[0];
  L.work = &s_work[0];
  const uint32_t nq = W.ctr[2 * QF];
  const bool dyn = K.V.on;
  // a wave-uniform loop (the fb frequencies are computed by the whole wave, wave_select_continuum_nu)
  for (uint32_t slot0 = blockIdx.x * blockDim.x + threadIdx.x;; slot0 += gridDim.x * blockDim.x) {
    uint32_t slot = slot0;
    if (dyn) {
      if (__builtin_amdgcn_readfirstlane(*(volatile uint32_t *)K.V.full)) break;
      slot = wave_reserve(&W.ctr[2 * QF + 1], true);
    }
    const bool have = slot < nq;
    if (!__any(have)) break;
    int32_t idx = -1;
    Pkt p;
    Tx x(K, L);
    MaEnd e{};
    FbReq fb;
    unsigned jumps = 0;
    if (have) {
      idx = W.q[QF][slot];
      pkt_load_finish(soa, n, idx, p);
      x.nts = nts;
      x.rng = artis_rng_init(K.R.seed, p.number, nts, K.R.rank);
      if (W.mf_rec) {
        const int4 pd = W.mf_rec[2 * (int64_t)slot], pj = W.mf_rec[2 * (int64_t)slot + 1];
        e = MaEnd{pd.x, pd.y, pd.z, pd.w};
        jumps = (unsigned)pj.x;
        x.rng.n = (uint32_t)pj.y;
      } else {
        x.rng.n = W.rng_n[idx];
        const int4 pd = W.pend[idx];
        e = MaEnd{pd.x, pd.y, pd.z, pd.w};
        jumps = W.pend_jumps[idx];
      }
      if (e.code == MA_END_FB) {  // ma_finish_fb's continuum and its first draw (select_continuum_nu's)
        const int uiu = K.T.level_ui[e.b];
        fb.want = true;
        fb.e = p.ma_element;
        fb.ion = uiu - K.T.elem_uniqueionoffset[p.ma_element] - 1;
        fb.lower = e.a;
        fb.upper = e.b - K.T.ion_uniqueleveloffset[uiu];
        fb.T_e = K.C.Te[cell_mgi(K, p.where)];
        fb.zrand = 1. - artis_rng_uniform(&x.rng);
      }
    }
    const double fb_nu = wave_select_continuum_nu(K, fb.want, fb.e, fb.ion, fb.lower, fb.upper, fb.T_e, fb.zrand, fbP);
    bool live = false;
    if (have) {
      const bool first = p.trueemissiontype < 0;
      ma_finish_inl(x, p, e, jumps, fb.want ? fb_nu : -1.);
      if (!W.mf_rec) W.pend[idx].x = 0;
      pkt_store_finish(soa, n, idx, p, e.code == MA_END_BB || e.code == MA_END_FB, first);
      W.rng_n[idx] = x.rng.n;
      live = x.ok && p.prop_time < t2;
    }
    wave_push(W, QR, live && p.type == ARTIS_TYPE_RPKT, idx);
    wave_push(W, QK, live && (p.type == ARTIS_TYPE_KPKT || p.type == ARTIS_TYPE_PRE_KPKT), idx);
  }
  block_counters_flush(K, s_ctr, s_work);
}

// pellets, gamma rays and non-thermal leptons (gamma.h): one packet per workitem, grid-stride over the G queue,
// each advanced until it becomes a k-packet (-> K queue), escapes or reaches t2.  Runs once per timestep before
// the r-packet / macro-atom / k-packet rounds (nothing on those paths turns back into this family).
__global__ __launch_bounds__(WAVE_BLOCK, 3) void k_gamma(const Ctx *__restrict__ ctxp, WaveState W, uint64_t *__restrict__ soa,
                                                      int64_t n, int nts, double t2) {
  CTX_IN_LDS(ctxp)
  __shared__ unsigned long long s_ctr[ARTIS_COUNTER_COUNT + 1];
  __shared__ unsigned long long s_work[ARTIS_WORK_COUNT];
  block_counters_init(s_ctr, s_work);
  LocalCounters L;
  L.ctr = &s_ctr[0];
  L.work = &s_work[0];
  const uint32_t nq = W.ctr[2 * QG];
  const uint32_t stride = gridDim.x * blockDim.x;
  // uniform trip count so the wave-aggregated queue appends see every lane of the wave
  const uint32_t nslots = (nq + stride - 1) / stride * stride;
  for (uint32_t slot = blockIdx.x * blockDim.x + threadIdx.x; slot < nslots; slot += stride) {
    bool toR = false, toM = false, toK = false;
    int32_t idx = -1;
    int m_where = 0, m_number = 0;  // the pre-ticket of a macro-atom (toM)
    uint32_t m_rng = 0;
    int4 m_b = make_int4(0, 0, 0, 0);
    if (slot < nq) {
      idx = W.q[QG][slot];
      Pkt p;
      pkt_load(soa, n, idx, p);
      PelletInfo pi;
      pellet_info_load(soa, n, idx, pi);
      Tx x(K, L);
      x.nts = nts;
      x.rng = artis_rng_init(K.R.seed, p.number, nts, K.R.rank);
      x.rng.n = W.rng_n[idx];
      int guard = 0;
      while (x.ok && is_gamma_family(p.type) && p.prop_time < t2) {
        do_gamma_family_step(x, p, pi, t2);
        if (++guard > 1000000) x.err(ERR_STUCK, p.number, 5);
      }
      pkt_store(soa, n, idx, p);
      W.rng_n[idx] = x.rng.n;
      if (x.ok && p.prop_time < t2) {
        toR = p.type == ARTIS_TYPE_RPKT;
        toM = p.type == ARTIS_TYPE_MA;
        toK = p.type == ARTIS_TYPE_KPKT || p.type == ARTIS_TYPE_PRE_KPKT;
      }
      m_where = p.where;
      m_number = p.number;
      m_rng = x.rng.n;
      m_b = ma_pre_activation(p.ma_element, p.ma_ion, p.ma_level);
    }
    wave_push(W, QR, toR, idx);
    wave_push_ma(W, toM, idx, m_where, m_number, m_rng, m_b, ma_push_bin(K, W, toM, m_where));
    wave_push(W, QK, toK, idx);
  }
  block_counters_flush(K, s_ctr, s_work);
}

// k-packets (rare): one packet per workitem, grid-stride
__global__ __launch_bounds__(WAVE_BLOCK) void k_kpkt(const Ctx *__restrict__ ctxp, WaveState W, uint64_t *__restrict__ soa, int64_t n,
                                                     int nts, double t2) {
  CTX_IN_LDS(ctxp)
  __shared__ unsigned long long s_ctr[ARTIS_COUNTER_COUNT + 1];
  __shared__ unsigned long long s_work[ARTIS_WORK_COUNT];
  __shared__ double s_fbP[WAVE_BLOCK / 64][WAVE_FB_MAXP + 1];  // the waves' fb running sums (wave_select_continuum_nu)
  lds_double *fbP = (lds_double *)&s_fbP[threadIdx.x >> 6][0];
  block_counters_init(s_ctr, s_work);
  LocalCounters L;
  L.ctr = &s_ctr[0];
  L.work = &s_work[0];
  const uint32_t nq = W.ctr[2 * QK];
  // with virtual packets the slots are taken a wave at a time from the fetch head, so that a full spawn buffer can
  // stop the launch with the untaken slots [head, nq) left for the resumed launch (engine.hip vpkt_drain).  The loop
  // is wave-uniform: an fb cooling emission's frequency is computed by the whole wave (wave_select_continuum_nu).
  const bool dyn = K.V.on;
  for (uint32_t slot0 = blockIdx.x * blockDim.x + threadIdx.x;; slot0 += gridDim.x * blockDim.x) {
    uint32_t slot = slot0;
    if (dyn) {
      if (__builtin_amdgcn_readfirstlane(*(volatile uint32_t *)K.V.full)) break;
      slot = wave_reserve(&W.ctr[2 * QK + 1], true);
    }
    const bool have = slot < nq;
    if (!__any(have)) break;
    int32_t idx = -1;
    Pkt p;
    Tx x(K, L);
    if (have) {
      idx = W.q[QK][slot];
      pkt_load(soa, n, idx, p);
      x.nts = nts;
      x.rng = artis_rng_init(K.R.seed, p.number, nts, K.R.rank);
      x.rng.n = W.rng_n[idx];
    }
    int guard = 0;
    while (true) {
      const bool kp = have && x.ok && (p.type == ARTIS_TYPE_KPKT || p.type == ARTIS_TYPE_PRE_KPKT) && p.prop_time < t2;
      if (!__any(kp)) break;
      FbReq fb;
      if (kp) {
        const int mgi = cell_mgi(K, p.where);
        if (p.type == ARTIS_TYPE_PRE_KPKT || K.C.thick[mgi] == 1)
          do_kpkt_bb(x, p);
        else
          do_kpkt(x, p, t2, &fb);
      }
      const double nu = wave_select_continuum_nu(K, fb.want, fb.e, fb.ion, fb.lower, fb.upper, fb.T_e, fb.zrand, fbP);
      if (fb.want) kpkt_fb_tail(x, p, fb.e, fb.ion, fb.lower, fb.upper, nu);
      if (kp && ++guard > 1000) x.err(ERR_STUCK, p.number, 4);
    }
    bool toR = false, toM = false;
    if (have) {
      pkt_store(soa, n, idx, p);
      W.rng_n[idx] = x.rng.n;
      toR = x.ok && p.prop_time < t2 && p.type == ARTIS_TYPE_RPKT;
      toM = x.ok && p.prop_time < t2 && p.type == ARTIS_TYPE_MA;
    }
    wave_push(W, QR, toR, idx);
    wave_push_ma(W, toM, idx, p.where, p.number, x.rng.n, ma_pre_activation(p.ma_element, p.ma_ion, p.ma_level),
                 ma_push_bin(K, W, toM, p.where));
  }
  block_counters_flush(K, s_ctr, s_work);
}

#endif
