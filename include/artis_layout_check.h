/*
 * artis_layout_check.h -- compile-time proof that artis_packet is the reference's `struct packet`
 * (packet.h:28-73; probed sizeof 304 and offsets in SURVEY.md §8(b)).  Include it from any translation unit
 * that hands packet arrays across the boundary (the host mirror does).
 */
#ifndef ARTIS_LAYOUT_CHECK_H
#define ARTIS_LAYOUT_CHECK_H

#include <stddef.h>

#include "artis_gpu.h"

#ifdef __cplusplus
#define ARTIS_STATIC_ASSERT(c, m) static_assert(c, m)
#else
#define ARTIS_STATIC_ASSERT(c, m) _Static_assert(c, m)
#endif

ARTIS_STATIC_ASSERT(sizeof(artis_packet) == 304, "struct packet is 304 bytes");
ARTIS_STATIC_ASSERT(offsetof(artis_packet, where) == 0, "where");
ARTIS_STATIC_ASSERT(offsetof(artis_packet, type) == 4, "type");
ARTIS_STATIC_ASSERT(offsetof(artis_packet, pos) == 24, "pos");
ARTIS_STATIC_ASSERT(offsetof(artis_packet, dir) == 48, "dir");
ARTIS_STATIC_ASSERT(offsetof(artis_packet, e_cmf) == 72, "e_cmf");
ARTIS_STATIC_ASSERT(offsetof(artis_packet, e_rf) == 80, "e_rf");
ARTIS_STATIC_ASSERT(offsetof(artis_packet, nu_cmf) == 88, "nu_cmf");
ARTIS_STATIC_ASSERT(offsetof(artis_packet, nu_rf) == 96, "nu_rf");
ARTIS_STATIC_ASSERT(offsetof(artis_packet, next_trans) == 104, "next_trans");
ARTIS_STATIC_ASSERT(offsetof(artis_packet, prop_time) == 144, "prop_time");
ARTIS_STATIC_ASSERT(offsetof(artis_packet, stokes) == 200, "stokes");
ARTIS_STATIC_ASSERT(offsetof(artis_packet, tdecay) == 248, "tdecay");
ARTIS_STATIC_ASSERT(offsetof(artis_packet, number) == 268, "number");
ARTIS_STATIC_ASSERT(offsetof(artis_packet, mastate) == 288, "mastate");

#endif
