/*
 * artis_rng.h -- counter-based per-packet random stream (Philox4x32-10, Salmon et al. SC'11).
 *
 * Replaces the reference's per-OpenMP-thread GSL ran3 generator (seeded pre_zseed + 13*rank + 17*tid,
 * input.cc:1908-1917) whose stream order depends on which thread ran which packet.  Here every packet owns
 * its stream, keyed by (seed, packet number) with counter (draw index, nts, rank), so any schedule -- one CPU
 * thread, 64 OpenMP threads, or 10^7 GPU workitems -- draws identical numbers for a packet.  This is what
 * makes per-packet parity between the oracle and the HIP engine possible.
 *
 * Draw semantics follow GSL: uniform() in [0,1) (gsl_rng_uniform) and uniform_pos() in (0,1)
 * (gsl_rng_uniform_pos, which redraws on 0).  53 random bits per draw.
 */
#ifndef ARTIS_RNG_H
#define ARTIS_RNG_H

#include <stdint.h>

#if defined(__HIPCC__)
#define ARTIS_HD __host__ __device__ __forceinline__
#else
#define ARTIS_HD inline
#endif

typedef struct artis_rng {
  uint32_t key0;   /* seed */
  uint32_t key1;   /* packet number */
  uint32_t nts;
  uint32_t rank;
  uint32_t n;      /* draws so far in this timestep */
} artis_rng;

ARTIS_HD uint32_t artis_mulhilo32(uint32_t a, uint32_t b, uint32_t *hi) {
  const uint64_t p = (uint64_t)a * (uint64_t)b;
  *hi = (uint32_t)(p >> 32);
  return (uint32_t)p;
}

ARTIS_HD void artis_philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
  for (int r = 0; r < 10; r++) {
    uint32_t hi0, hi1;
    const uint32_t lo0 = artis_mulhilo32(0xD2511F53u, c[0], &hi0);
    const uint32_t lo1 = artis_mulhilo32(0xCD9E8D57u, c[2], &hi1);
    const uint32_t n0 = hi1 ^ c[1] ^ k0;
    const uint32_t n2 = hi0 ^ c[3] ^ k1;
    c[0] = n0;
    c[1] = lo1;
    c[2] = n2;
    c[3] = lo0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}

ARTIS_HD artis_rng artis_rng_init(uint32_t seed, int32_t packet_number, int32_t nts, int32_t rank) {
  artis_rng s;
  s.key0 = seed;
  s.key1 = (uint32_t)packet_number;
  s.nts = (uint32_t)nts;
  s.rank = (uint32_t)rank;
  s.n = 0;
  return s;
}

/* 53-bit integer of draw number s->n, then advance */
ARTIS_HD uint64_t artis_rng_next53(artis_rng *s) {
  uint32_t c[4] = {s->n, 0x41525453u, s->nts, s->rank};
  artis_philox4x32_10(c, s->key0, s->key1);
  s->n++;
  const uint64_t x = ((uint64_t)c[1] << 32) | (uint64_t)c[0];
  return x >> 11;
}

/* The two draws of one macro-atom jump (do_macroatom, macroatom.cc:416-901: the action, then the transition within
 * it) at counters n and n + 1 come from one Philox block, block n: the action draw is words 0-1 (what
 * artis_rng_uniform returns at counter n), the transition draw words 2-3.  Block n + 1 is never evaluated for a jump:
 * one Philox evaluation per jump instead of two, on the engine's busiest kernel (part of deviation D1: the stream is
 * this library's definition, the same on both sides).  The caller advances s->n over the draws it consumes, as with
 * artis_rng_uniform; a jump that consumes only the action draw leaves counter n + 1 to the next draw. */
ARTIS_HD void artis_rng_jump_words(const artis_rng *s, uint32_t w[4]) {
  w[0] = s->n;
  w[1] = 0x41525453u;
  w[2] = s->nts;
  w[3] = s->rank;
  artis_philox4x32_10(w, s->key0, s->key1);
}
/* the uniform draw of words (lo, hi) of a block: the top 53 bits over 2^53 */
ARTIS_HD double artis_rng_word_unit(uint32_t lo, uint32_t hi) {
  return (double)((((uint64_t)hi << 32) | (uint64_t)lo) >> 11) * (1.0 / 9007199254740992.0);
}
ARTIS_HD void artis_rng_jump_pair(const artis_rng *s, double *z1, double *z2) {
  uint32_t c[4];
  artis_rng_jump_words(s, c);
  *z1 = artis_rng_word_unit(c[0], c[1]);
  *z2 = artis_rng_word_unit(c[2], c[3]);
}

/* gsl_rng_uniform: [0,1) */
ARTIS_HD double artis_rng_uniform(artis_rng *s) { return (double)artis_rng_next53(s) * (1.0 / 9007199254740992.0); }

/* gsl_rng_uniform_pos: (0,1) */
ARTIS_HD double artis_rng_uniform_pos(artis_rng *s) {
  uint64_t x;
  do {
    x = artis_rng_next53(s);
  } while (x == 0);
  return (double)x * (1.0 / 9007199254740992.0);
}

#endif /* ARTIS_RNG_H */
