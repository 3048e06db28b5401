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
 * and the run inputs the reference reads before the timestep loop:
 *   input.txt              read_parameterfile  input.cc:1874-2140 (24 positional lines, '#' comments skipped)
 *   model.txt              read_1d_model grid.cc:1228-1370 / read_3d_model grid.cc:1459-1600
 *                          (+ read_model_headerline grid.cc:1080-1156, read_2d3d_modelradioabundanceline 1158-1226)
 *   abundances.txt         abundances_read     grid.cc:1007-1073
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

/* input.txt (read_parameterfile, input.cc:1874-2140).  Values as the reference stores them: times in days as
 * given (globals::tmin = tmin_days * DAY), do_r_lc / do_rlc_est derived from the r-light-curve line as
 * input.cc:1976-1979, syn_dir normalised (zero vector kept as zero: the reference then draws a random one). */
typedef struct artis_input_params {
  uint32_t pre_zseed;          /* line 1 (> 0: the seed) */
  int32_t ntstep;              /* line 2 */
  int32_t itstep, ftstep;      /* line 3 */
  double tmin_days, tmax_days; /* line 4 */
  double nusyn_min_mev, nusyn_max_mev; /* line 5 */
  int32_t nsyn_time;           /* line 6 */
  double syn_time_start_days, syn_time_dlog; /* line 7 */
  int32_t model_type;          /* line 8: 1 RHO_1D_READ, 2 RHO_2D_READ, 3 RHO_3D_READ */
  int32_t rlc_mode;            /* line 9 as read (0..4) */
  int32_t do_r_lc, do_rlc_est; /* derived from line 9 (input.cc:1976-1979) */
  int32_t n_out_it;            /* line 10 */
  double clight_factor;        /* line 11 (must be 1) */
  double gamma_grey;           /* line 12 */
  double syn_dir[3];           /* line 13 */
  int32_t opacity_case;        /* line 14 */
  double rho_crit_para;        /* line 15 */
  int32_t debug_packet;        /* line 16 */
  int32_t continued_from_saved;/* line 17 */
  double rfcut_angstroms;      /* line 18 */
  int32_t num_lte_timesteps;   /* line 19 */
  double cell_is_optically_thick; int32_t num_grey_timesteps; /* line 20 */
  int32_t max_bf_continua;     /* line 21 (-1 read as unlimited, stored as 1000000 as input.cc:2094-2096) */
  int32_t nprocs_exspec;       /* line 22 */
  int32_t do_emission_res;     /* line 23 */
  double kpktdiffusion_timescale; int32_t n_kpktdiffusion_timesteps; /* line 24 */
} artis_input_params;
int artis_read_input_file(const char *filename, artis_input_params *out);

/* model.txt for model_type 1 (1D shells) or 3 (3D cuboid; 2D is rejected).  Arrays are allocated by the reader
 * and released by artis_free_model.  Densities at t_model as in the file (the reference scales them by
 * (t_model/tmin)^3 afterwards, grid.cc:1302, 1565); radioactive mass fractions from the first 5 or 7 abundance
 * columns; custom header columns (X_<nuclide>, cellYe, q, tracercount; grid.cc:1080-1156) are parsed and
 * counted but not stored (the engine does not propagate decay chains). */
typedef struct artis_ejecta_model {
  int32_t model_type;
  int32_t npts_model;
  int32_t ncoord_model[3];   /* 1D {npts,1,1}; 3D cube-root of npts on each axis (grid.cc:1475) */
  double t_model;            /* [s] */
  double vmax;               /* [cm/s]: 1D outer velocity of the last shell (grid.cc:1369); 3D header line 3 */
  double *vout;              /* [npts] 1D outer shell velocities [cm/s]; NULL for 3D */
  double *rho_model;         /* [npts] [g/cm^3] at t_model */
  double *ffegrp, *x_ni56, *x_co56, *x_fe52, *x_cr48, *x_ni57, *x_co57; /* [npts] */
  float *pos_model;          /* [npts * 3] 3D cell positions as given (x,y,z columns), NULL for 1D */
  int32_t n_custom_columns;
  int32_t posorder_zyx;      /* 3D: the positions match z-y-x column order (grid.cc:1586-1592) */
} artis_ejecta_model;
int artis_read_model(const char *filename, int model_type, artis_ejecta_model *out);
void artis_free_model(artis_ejecta_model *m);

/* abundances.txt: one row per model cell, "cellnumber X(Z=1) X(Z=2) ...", normalised to the row sum unless the
 * model is 3D (grid.cc:1038-1058).  Writes elem_abund[mgi * nelements + element] for the given atomic numbers. */
int artis_read_abundances(const char *filename, int npts_model, int model_type, int nelements,
                          const int32_t *anumber, float *elem_abund);

/* Spectrum and light-curve writers (the formats of spectrum.cc:172-298 write_spectrum / write_specpol and
 * light_curve.cc:9-32 write_light_curve), for the arrays artis_gpu_spectra fills (include/artis_gpu.h):
 *   spec.out: "0 t_mid/DAY ..." then per frequency bin "nu_mid flux(t) ..."; nu_mid from the float bin edges
 *     of init_spectra (spectrum.cc:495-500);
 *   emission.out / emissiontrue.out / absorption.out: per (frequency bin, timestep) one row of proccount
 *     (ioncount) columns;
 *   specpol.out: header with the timestep list three times, then per bin "nu_mid I(t)... Q(t)... U(t)...";
 *     emissionpol.out / absorptionpol.out rows in the order I, Q, U per bin;
 *   light_curve.out: "t_mid/DAY lum/LSUN lumcmf/LSUN" rows, then (abin -1) "t_mid/DAY gamma_dep/LSUN/width
 *     cmf_lum/width/LSUN" rows.
 * Every value printed with "%g " as the reference does.  NULL emission filenames / arrays skip those files.
 * 0 on success, -1 when a file cannot be written. */
int artis_write_spectrum(const char *spec_filename, const char *emission_filename, const char *trueemission_filename,
                         const char *absorption_filename, int ntstep, int numtimesteps, const double *ts_mid,
                         int nnubins, double nu_min, double nu_max, int proccount, int ioncount, const double *flux,
                         const double *emission, const double *trueemission, const double *absorption);
int artis_write_specpol(const char *specpol_filename, const char *emission_filename, const char *absorption_filename,
                        int ntstep, const double *ts_mid, int nnubins, double nu_min, double nu_max, int proccount,
                        int ioncount, const double *stokes_flux, const double *stokes_emission,
                        const double *stokes_absorption);
int artis_write_light_curve(const char *lc_filename, int abin, int numtimesteps, const double *ts_mid,
                            const double *ts_width, const double *lc_lum, const double *lc_lumcmf,
                            const double *gamma_dep, const double *cmf_lum);

/* The Spencer-Fano data nonthermal::init reads (nonthermal.cc:183-437) from directory dir: binding_energies.txt
 * (read_binding_energies), collion.txt (read_collion_data: the rows of the included ions -- elements anumber[e]
 * with ion stages ionstage0[e] .. ionstage0[e] + nions[e] - 1 -- in file order) and auger-km1993-table2.txt
 * (read_auger_data: Auger-electron probabilities and mean energies, g-weighted over the X-ray subshells that map to
 * each row's n, l).  Fills out->shells (whose arrays out owns) with the energy grid sfpts / sf_emin / sf_emax.
 * Release with artis_free_nt_data. */
typedef struct artis_nt_data {
  artis_nt_shells shells;
  void *storage;
} artis_nt_data;
int artis_read_nt_data(const char *dir, int nelements, const int32_t *anumber, const int32_t *ionstage0,
                       const int32_t *nions, int sfpts, double sf_emin, double sf_emax, artis_nt_data *out);
void artis_free_nt_data(artis_nt_data *d);

#ifdef __cplusplus
}
#endif

#endif /* ARTIS_IO_H */
