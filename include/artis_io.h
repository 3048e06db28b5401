/*
 * artis_io.h -- the reference's packet and virtual-packet file formats, for the host around the engine.
 *
 * The engine hands packets back in the reference's 304-byte layout (artis_gpu.h), so the reference's own
 * writers keep working on them; these functions restate the formats for a host that does not link the
 * reference (tests, tools/, artis_gpu_driver).  Every format is the reference's byte for byte:
 *   packets00_RRRR.out     write_packets   packet.cc:152-196 (text, printf %d / %g / %lg fields)
 *                          read_packets    packet.cc:211-290
 *   packets_RRRR_tsN.tmp   write_temp_packetsfile sn3d.cc:387-398 / read_temp_packetsfile packet.cc:198-209
 *   vspecpol_*.out / .tmp  write_vspecpol  vpkt.cc:445-483 / read_vspecpol vpkt.cc:485-545
 *   vpkt_grid_*.out / .tmp write_vpkt_grid vpkt.cc:629-646 / read_vpkt_grid vpkt.cc:648-665
 * Returns 0, or a negative artis_status (ARTIS_ERR_BAD_ARGUMENT for an unreadable / short file).
 */
#ifndef ARTIS_IO_H
#define ARTIS_IO_H

#include "artis_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

int artis_write_packets(const char *filename, const artis_packet *pkts, int npkts);
int artis_read_packets(const char *filename, artis_packet *pkts, int npkts);
/* dir may be NULL (current directory); file name packets_%.4d_ts%d.tmp of my_rank and timestep */
int artis_write_temp_packetsfile(const char *dir, int timestep, int my_rank, const artis_packet *pkts, int npkts);
int artis_read_temp_packetsfile(const char *dir, int timestep, int my_rank, artis_packet *pkts, int npkts);

/* vstokes_i/q/u of *r in the artis_vpkt_result layout; read fills them (overwrites) */
int artis_write_vspecpol(const char *filename, const artis_vpkt_params *p, const artis_vpkt_result *r);
int artis_read_vspecpol(const char *filename, const artis_vpkt_params *p, artis_vpkt_result *r);
/* vgrid_i/q/u of *r; vmax = globals::vmax (grid.cc), the extent of the velocity map (vpkt.cc:548-574) */
int artis_write_vpkt_grid(const char *filename, const artis_vpkt_params *p, double vmax, const artis_vpkt_result *r);
int artis_read_vpkt_grid(const char *filename, const artis_vpkt_params *p, artis_vpkt_result *r);

#ifdef __cplusplus
}
#endif

#endif /* ARTIS_IO_H */
