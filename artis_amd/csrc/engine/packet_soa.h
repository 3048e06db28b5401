// packet_soa.h -- register image of one packet and its load/store to the packet store in HBM (engine_dev.h).
// Word map = byte offsets of the reference `struct packet` (packet.h:28-73) divided by 8.
//
// Layout: the 38 words of every packet are grouped by how the event-queue kernels touch them --
//   hot  (16 words, 128 B = one cache line per packet): what every r-packet step reads and writes
//   cold (20 words in a 24-word, 192-byte record of three 64-byte sectors, each written by one kind of event):
//     sector 0 (words 19, 21-24, 36, 37, 20): the absorption record and macro-atom state a line absorption writes
//              (k_rpkt), with the trueemission words beside them;
//     sector 1 (words 14-17, 25-28) and the first two of sector 2 (29, 30): the emission record, Stokes vector and
//              polarisation direction a deactivation writes (k_ma_finish);
//     sector 2 also holds the escape record (32) and word 35.
//   rest (2 words): tdecay and the pellet bookkeeping, never touched by this path
// each group stored packet-major ([group base + packet * group width + slot]).  The queues hand packets to
// kernels in arbitrary order, so a word-major (SoA) layout would cost one 128-byte line per 8-byte word;
// grouped, a packet's hot state is one line, and an event's cold writes fill one sector instead of touching
// three lines of a 160-byte record (round 6: k_rpkt wrote 0.80 GB per launch for the absorption record alone,
// profiles/r6h_write_diag.txt).
#ifndef ARTIS_PACKET_SOA_H
#define ARTIS_PACKET_SOA_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "engine_dev.h"

#define PKT_COLD_WIDTH 24
#define PKT_STORE_WORDS (16 + PKT_COLD_WIDTH + 2)  // words of the packet store per packet (PKT_WORDS of payload)

// word -> group (0 hot, 1 cold, 2 rest) and slot within the group; constant-folded for literal words
__host__ __device__ constexpr int pkt_word_group(int w) {
  return (w == 31 || w == 34) ? 2 : ((w >= 14 && w <= 17) || (w >= 19 && w <= 30) || w == 32 || w >= 35) ? 1 : 0;
}
__host__ __device__ constexpr int pkt_word_slot(int w) {
  return w <= 13 ? w : w == 18 ? 14 : w == 33 ? 15                              // hot
       : w == 19 ? 0 : (w >= 21 && w <= 24) ? w - 20 : w == 36 ? 5 : w == 37 ? 6  // cold sector 0
       : w == 20 ? 7
       : (w >= 14 && w <= 17) ? w - 6 : (w >= 25 && w <= 28) ? w - 13           // cold sector 1
       : (w == 29 || w == 30) ? w - 13 : w == 32 ? 18 : w == 35 ? 19             // cold sector 2
       : w == 31 ? 0 : 1;                                                       // rest: 31, 34
}
__host__ __device__ constexpr int64_t pkt_word_index(int64_t n, int64_t i, int w) {
  return pkt_word_group(w) == 0   ? i * 16 + pkt_word_slot(w)
         : pkt_word_group(w) == 1 ? 16 * n + i * PKT_COLD_WIDTH + pkt_word_slot(w)
                                  : (16 + PKT_COLD_WIDTH) * n + i * 2 + pkt_word_slot(w);
}
#define PW(n, i, w) pkt_word_index((n), (i), (w))

struct Pkt {
  int32_t where, type, last_cross, interactions, nscatterings, last_event;
  double pos[3], dir[3];
  double e_cmf, e_rf, nu_cmf, nu_rf;
  int32_t next_trans, emissiontype;
  double em_pos[3];
  int32_t em_time, pad0;
  double prop_time;
  int32_t absorptiontype, trueemissiontype, trueem_time, pad1;
  double absorptionfreq;
  double absorptiondir[3], stokes[3], pol_dir[3];
  int32_t escape_type, escape_time, scat_count, number;
  int32_t pellet_nucindex;
  float trueemissionvelocity;
  int32_t ma_element, ma_ion, ma_level, ma_activatingline;
};

__device__ __forceinline__ uint64_t pack2(int32_t lo, int32_t hi) {
  return (uint64_t)(uint32_t)lo | ((uint64_t)(uint32_t)hi << 32);
}
__device__ __forceinline__ int32_t lo32(uint64_t w) { return (int32_t)(uint32_t)w; }
__device__ __forceinline__ int32_t hi32(uint64_t w) { return (int32_t)(uint32_t)(w >> 32); }
__device__ __forceinline__ double asd(uint64_t w) { return __longlong_as_double((long long)w); }
__device__ __forceinline__ uint64_t asw(double d) { return (uint64_t)__double_as_longlong(d); }

__device__ __forceinline__ void pkt_load(const uint64_t *__restrict__ soa, int64_t n, int64_t i, Pkt &p) {
#define W(k) soa[pkt_word_index(n, i, (k))]
  uint64_t w;
  w = W(0);
  p.where = lo32(w);
  p.type = hi32(w);
  w = W(1);
  p.last_cross = lo32(w);
  p.interactions = hi32(w);
  w = W(2);
  p.nscatterings = lo32(w);
  p.last_event = hi32(w);
  for (int d = 0; d < 3; d++) p.pos[d] = asd(W(3 + d));
  for (int d = 0; d < 3; d++) p.dir[d] = asd(W(6 + d));
  p.e_cmf = asd(W(9));
  p.e_rf = asd(W(10));
  p.nu_cmf = asd(W(11));
  p.nu_rf = asd(W(12));
  w = W(13);
  p.next_trans = lo32(w);
  p.emissiontype = hi32(w);
  for (int d = 0; d < 3; d++) p.em_pos[d] = asd(W(14 + d));
  w = W(17);
  p.em_time = lo32(w);
  p.pad0 = hi32(w);
  p.prop_time = asd(W(18));
  w = W(19);
  p.absorptiontype = lo32(w);
  p.trueemissiontype = hi32(w);
  w = W(20);
  p.trueem_time = lo32(w);
  p.pad1 = hi32(w);
  p.absorptionfreq = asd(W(21));
  for (int d = 0; d < 3; d++) p.absorptiondir[d] = asd(W(22 + d));
  for (int d = 0; d < 3; d++) p.stokes[d] = asd(W(25 + d));
  for (int d = 0; d < 3; d++) p.pol_dir[d] = asd(W(28 + d));
  w = W(32);
  p.escape_type = lo32(w);
  p.escape_time = hi32(w);
  w = W(33);
  p.scat_count = lo32(w);
  p.number = hi32(w);
  w = W(35);
  p.pellet_nucindex = lo32(w);
  p.trueemissionvelocity = __int_as_float(hi32(w));
  w = W(36);
  p.ma_element = lo32(w);
  p.ma_ion = hi32(w);
  w = W(37);
  p.ma_level = lo32(w);
  p.ma_activatingline = hi32(w);
#undef W
}

// words 31 (tdecay) and 34 (pellet bookkeeping) are never written by the transport path
__device__ __forceinline__ void pkt_store(uint64_t *__restrict__ soa, int64_t n, int64_t i, const Pkt &p) {
#define W(k) soa[pkt_word_index(n, i, (k))]
  W(0) = pack2(p.where, p.type);
  W(1) = pack2(p.last_cross, p.interactions);
  W(2) = pack2(p.nscatterings, p.last_event);
  for (int d = 0; d < 3; d++) W(3 + d) = asw(p.pos[d]);
  for (int d = 0; d < 3; d++) W(6 + d) = asw(p.dir[d]);
  W(9) = asw(p.e_cmf);
  W(10) = asw(p.e_rf);
  W(11) = asw(p.nu_cmf);
  W(12) = asw(p.nu_rf);
  W(13) = pack2(p.next_trans, p.emissiontype);
  for (int d = 0; d < 3; d++) W(14 + d) = asw(p.em_pos[d]);
  W(17) = pack2(p.em_time, p.pad0);
  W(18) = asw(p.prop_time);
  W(19) = pack2(p.absorptiontype, p.trueemissiontype);
  W(20) = pack2(p.trueem_time, p.pad1);
  W(21) = asw(p.absorptionfreq);
  for (int d = 0; d < 3; d++) W(22 + d) = asw(p.absorptiondir[d]);
  for (int d = 0; d < 3; d++) W(25 + d) = asw(p.stokes[d]);
  for (int d = 0; d < 3; d++) W(28 + d) = asw(p.pol_dir[d]);
  W(32) = pack2(p.escape_type, p.escape_time);
  W(33) = pack2(p.scat_count, p.number);
  W(35) = pack2(p.pellet_nucindex, __float_as_int(p.trueemissionvelocity));
  W(36) = pack2(p.ma_element, p.ma_ion);
  W(37) = pack2(p.ma_level, p.ma_activatingline);
#undef W
}

// Hot/cold split for the r-packet kernel.  Hot words are what the propagation step reads; cold words
// (emission / absorption bookkeeping, polarisation, escape record, macro-atom state) are only read by the rare
// event code, which runs on a copy assembled from the hot registers plus the cold words in HBM.
__device__ __forceinline__ void pkt_load_hot(const uint64_t *__restrict__ soa, int64_t n, int64_t i, Pkt &p) {
#define W(k) soa[pkt_word_index(n, i, (k))]
  uint64_t w;
  w = W(0);
  p.where = lo32(w);
  p.type = hi32(w);
  w = W(1);
  p.last_cross = lo32(w);
  p.interactions = hi32(w);
  w = W(2);
  p.nscatterings = lo32(w);
  p.last_event = hi32(w);
  for (int d = 0; d < 3; d++) p.pos[d] = asd(W(3 + d));
  for (int d = 0; d < 3; d++) p.dir[d] = asd(W(6 + d));
  p.e_cmf = asd(W(9));
  p.e_rf = asd(W(10));
  p.nu_cmf = asd(W(11));
  p.nu_rf = asd(W(12));
  w = W(13);
  p.next_trans = lo32(w);
  p.emissiontype = hi32(w);
  p.prop_time = asd(W(18));
  w = W(33);
  p.scat_count = lo32(w);
  p.number = hi32(w);
#undef W
}
__device__ __forceinline__ void pkt_store_hot(uint64_t *__restrict__ soa, int64_t n, int64_t i, const Pkt &p) {
#define W(k) soa[pkt_word_index(n, i, (k))]
  W(0) = pack2(p.where, p.type);
  W(1) = pack2(p.last_cross, p.interactions);
  W(2) = pack2(p.nscatterings, p.last_event);
  for (int d = 0; d < 3; d++) W(3 + d) = asw(p.pos[d]);
  for (int d = 0; d < 3; d++) W(6 + d) = asw(p.dir[d]);
  W(9) = asw(p.e_cmf);
  W(10) = asw(p.e_rf);
  W(11) = asw(p.nu_cmf);
  W(12) = asw(p.nu_rf);
  W(13) = pack2(p.next_trans, p.emissiontype);
  W(18) = asw(p.prop_time);
  W(33) = pack2(p.scat_count, p.number);
#undef W
}
__device__ __forceinline__ void pkt_load_cold(const uint64_t *__restrict__ soa, int64_t n, int64_t i, Pkt &p) {
#define W(k) soa[pkt_word_index(n, i, (k))]
  uint64_t w;
  for (int d = 0; d < 3; d++) p.em_pos[d] = asd(W(14 + d));
  w = W(17);
  p.em_time = lo32(w);
  p.pad0 = hi32(w);
  w = W(19);
  p.absorptiontype = lo32(w);
  p.trueemissiontype = hi32(w);
  w = W(20);
  p.trueem_time = lo32(w);
  p.pad1 = hi32(w);
  p.absorptionfreq = asd(W(21));
  for (int d = 0; d < 3; d++) p.absorptiondir[d] = asd(W(22 + d));
  for (int d = 0; d < 3; d++) p.stokes[d] = asd(W(25 + d));
  for (int d = 0; d < 3; d++) p.pol_dir[d] = asd(W(28 + d));
  w = W(32);
  p.escape_type = lo32(w);
  p.escape_time = hi32(w);
  w = W(35);
  p.pellet_nucindex = lo32(w);
  p.trueemissionvelocity = __int_as_float(hi32(w));
  w = W(36);
  p.ma_element = lo32(w);
  p.ma_ion = hi32(w);
  w = W(37);
  p.ma_level = lo32(w);
  p.ma_activatingline = hi32(w);
#undef W
}
__device__ __forceinline__ void pkt_store_cold(uint64_t *__restrict__ soa, int64_t n, int64_t i, const Pkt &p) {
#define W(k) soa[pkt_word_index(n, i, (k))]
  for (int d = 0; d < 3; d++) W(14 + d) = asw(p.em_pos[d]);
  W(17) = pack2(p.em_time, p.pad0);
  W(19) = pack2(p.absorptiontype, p.trueemissiontype);
  W(20) = pack2(p.trueem_time, p.pad1);
  W(21) = asw(p.absorptionfreq);
  for (int d = 0; d < 3; d++) W(22 + d) = asw(p.absorptiondir[d]);
  for (int d = 0; d < 3; d++) W(25 + d) = asw(p.stokes[d]);
  for (int d = 0; d < 3; d++) W(28 + d) = asw(p.pol_dir[d]);
  W(32) = pack2(p.escape_type, p.escape_time);
  W(35) = pack2(p.pellet_nucindex, __float_as_int(p.trueemissionvelocity));
  W(36) = pack2(p.ma_element, p.ma_ion);
  W(37) = pack2(p.ma_level, p.ma_activatingline);
#undef W
}
// k_ma_finish (a macro-atom deactivation): the hot line and what the deactivation reads of sector 0 (the macro-atom
// state, trueemissiontype); a packet's first deactivation also reads the emission record and trueemission words it
// turns into the trueemission record (macroatom.cc:475-482).  The other cold fields stay unread and unwritten.
__device__ __forceinline__ void pkt_load_finish(const uint64_t *__restrict__ soa, int64_t n, int64_t i, Pkt &p) {
#define W(k) soa[pkt_word_index(n, i, (k))]
  pkt_load_hot(soa, n, i, p);
  uint64_t w = W(19);
  p.absorptiontype = lo32(w);
  p.trueemissiontype = hi32(w);
  w = W(36);
  p.ma_element = lo32(w);
  p.ma_ion = hi32(w);
  w = W(37);
  p.ma_level = lo32(w);
  p.ma_activatingline = hi32(w);
  if (p.trueemissiontype < 0) {
    for (int d = 0; d < 3; d++) p.em_pos[d] = asd(W(14 + d));
    w = W(17);
    p.em_time = lo32(w);
    p.pad0 = hi32(w);
    w = W(20);
    p.trueem_time = lo32(w);
    p.pad1 = hi32(w);
    w = W(35);
    p.pellet_nucindex = lo32(w);
    p.trueemissionvelocity = __int_as_float(hi32(w));
  }
#undef W
}
// emitted: an r-packet left the deactivation (bb / fb: emission record, Stokes vector, polarisation direction);
// first: the packet's first deactivation (pkt_load_finish read the trueemission words)
__device__ __forceinline__ void pkt_store_finish(uint64_t *__restrict__ soa, int64_t n, int64_t i, const Pkt &p,
                                                 bool emitted, bool first) {
#define W(k) soa[pkt_word_index(n, i, (k))]
  pkt_store_hot(soa, n, i, p);
  if (emitted) {
    for (int d = 0; d < 3; d++) W(14 + d) = asw(p.em_pos[d]);
    reinterpret_cast<int32_t *>(&W(17))[0] = p.em_time;  // (the word's upper half is padding: left as it is)
    for (int d = 0; d < 3; d++) W(25 + d) = asw(p.stokes[d]);
    for (int d = 0; d < 3; d++) W(28 + d) = asw(p.pol_dir[d]);
  }
  if (first) {
    W(19) = pack2(p.absorptiontype, p.trueemissiontype);
    W(20) = pack2(p.trueem_time, p.pad1);
    W(35) = pack2(p.pellet_nucindex, __float_as_int(p.trueemissionvelocity));
  }
#undef W
}

// hot fields only (the cold ones of `dst` are left as they are)
__device__ __forceinline__ void pkt_copy_hot(Pkt &dst, const Pkt &src) {
  dst.where = src.where;
  dst.type = src.type;
  dst.last_cross = src.last_cross;
  dst.interactions = src.interactions;
  dst.nscatterings = src.nscatterings;
  dst.last_event = src.last_event;
  for (int d = 0; d < 3; d++) {
    dst.pos[d] = src.pos[d];
    dst.dir[d] = src.dir[d];
  }
  dst.e_cmf = src.e_cmf;
  dst.e_rf = src.e_rf;
  dst.nu_cmf = src.nu_cmf;
  dst.nu_rf = src.nu_rf;
  dst.next_trans = src.next_trans;
  dst.emissiontype = src.emissiontype;
  dst.prop_time = src.prop_time;
  dst.scat_count = src.scat_count;
  dst.number = src.number;
}

#endif
