/*
 * model_synth.h -- synthetic ARTIS model: atomic data, propagation grid, per-timestep LTE cell state and
 * initial r-packets.  Test / bench infrastructure: it produces the frozen inputs that the reference's
 * input() + grid_init() + update_grid() hand to update_packets; it is not the hot
 * path and is not timed.  The atomic-data and model shapes follow SURVEY.md §8(d).
 */
#ifndef ARTIS_MODEL_SYNTH_H
#define ARTIS_MODEL_SYNTH_H

#include "artis_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct artis_synth_config {
  int32_t ngrid_1d;          /* uniform cuboid grid cells per axis (50 for the bench) */
  int32_t nshells_1d;        /* >0: 1D model with this many shells mapped onto the cuboid (map_1dmodeltogrid);
                                0: 3D model, one model cell per propagation cell (map_3dmodeltogrid) */
  int32_t nlevels_per_ion;   /* levels of each non-top ion */
  int32_t n_ionising;        /* levels with a bf continuum per non-top ion */
  int32_t max_lines;         /* cap on the line count (1e5 for the bench) */
  int32_t line_window;       /* each level has lines down to this many nearest lower levels ... */
  int32_t n_resonance;       /* ... and to the lowest n_resonance levels */
  int32_t ntstep;
  double tmin_days, tmax_days;
  double vmax;               /* cm/s */
  double mass_msun;          /* ejecta mass of the exponential profile */
  double v_e;                /* e-folding velocity of rho(v) */
  double T0;                 /* T(v) = T0 * (1 + 0.5 exp(-v / 5e8)) */
  int32_t n_tclasses;        /* temperature quantisation for the cooling-rate stand-in */
  uint64_t seed;
  double ionpot_scale;       /* scales every ionisation potential (test configs with bf-active continua); 0 = 1 */
  double thick_tau;          /* >0: cells whose grey optical depth across the cell exceeds this are "thick"
                                (input.txt cell_is_optically_thick, update_grid.cc); 0: none */
  int32_t relativistic;      /* USE_RELATIVISTIC_DOPPLER_SHIFT of the run parameters */
  int32_t instant_particle_deposition; /* INSTANT_PARTICLE_DEPOSITION (default 1, artisoptions_classic.h:222) */
  int32_t n_kpktdiffusion_timesteps;   /* input.txt "kpktdiffusion_timescale n_kpktdiffusion_timesteps"; the  */
  double kpktdiffusion_timescale;      /* reference test inputs use 0.001 1000 (default here: 0 0)         */
  int32_t excitation_te;     /* run parameter excitation_temperature: 0 T_J (classic), 1 T_e (kilonova, nebular) */
  double tj_scale;           /* T_J = tj_scale * T_e in the cell-state stand-in (0 = 1: T_J == T_e, as in the LTE
                                timesteps, update_grid.cc:1111-1114) */
  /* the nebular options (artisoptions_nltenebular.h): NLTE + superlevel populations, the binned radiation field,
     detailed bf estimators, NO_LUT photoionisation / bf-heating, non-thermal ionisation with Auger electrons,
     MINPOP 1e-40, NU_MIN_R 1e13, T_e excitation.  The update_grid outputs these read (NLTE populations, bin fits,
     normalised bf-rate estimators, the Spencer-Fano solution's rates and Auger fractions) are stand-ins drawn
     around the LTE state. */
  int32_t nebular;
  int32_t nlte_level_max;    /* LEVEL_IS_NLTE: levels 1..nlte_level_max of every ion are NLTE (default 80) */
  int32_t radfield_nbins;    /* RADFIELDBINCOUNT (default 256) */
  int32_t first_nlte_radfield_timestep;  /* FIRST_NLTE_RADFIELD_TIMESTEP (default 12) */
  int32_t detailed_bf_usefromtimestep;   /* DETAILED_BF_ESTIMATORS_USEFROMTIMESTEP (default 13) */
  double minpop;             /* MINPOP (0: 1e-30 classic, 1e-40 nebular) */
  double nu_min_r, nu_max_r; /* NU_MIN_R / NU_MAX_R (0: 1e14 / 5e15 classic; nebular 1e13 / 5e15) */
  int32_t grid_spherical;    /* 1D models only: GRID_SPHERICAL1D propagation grid, one radial cell per shell
                                (spherical1d_grid_setup, grid.cc:2104-2131) instead of the shells mapped onto the
                                ngrid_1d^3 cuboid (map_1dmodeltogrid) */
} artis_synth_config;

typedef struct artis_model artis_model;

void artis_synth_default_config(artis_synth_config *cfg);
artis_model *artis_model_synth(const artis_synth_config *cfg);
/* The reference's own run inputs: input.txt (times, seed, run switches), model.txt (1D or 3D) and
 * abundances.txt (Fe/Co/Ni mass fractions), read by include/artis_io.h; the atomic data stay synthetic (cfg),
 * cfg->ngrid_1d is CUBOID_NCOORDGRID for 1D models.  NULL on a malformed file. */
artis_model *artis_model_from_files(const artis_synth_config *cfg, const char *input_txt, const char *model_txt,
                                    const char *abundances_txt);
void artis_model_free(artis_model *m);

const artis_atomic_tables *artis_model_atomic(const artis_model *m);
const artis_geometry *artis_model_geometry(const artis_model *m);
const artis_cell_state *artis_model_cellstate(const artis_model *m);
/* bf-heating LUT and per-ion Alpha_sp of the model (update_grid's thermal balance, artis_gpu_solve_temperatures) */
const artis_te_tables *artis_model_te_tables(const artis_model *m);
void artis_model_run_params(const artis_model *m, artis_run_params *out);

/* LTE update_grid stand-in for timestep nts (densities scaled to ts_mid[nts]). */
int artis_model_set_timestep(artis_model *m, int nts);
// update_grid's host bookkeeping at timestep nts (density, grey opacity, thick flag); the rest of the cell state is
// left as it is
int artis_model_advance(artis_model *m, int nts);

/* Initial r-packets at the start of timestep nts: cell ~ rho*vol, isotropic direction, nu_cmf ~ Planck(T_e)
 * within [NU_MIN_R, NU_MAX_R], equal e_cmf (SURVEY.md §8(d) "pure r-packet benchmark"). */
int artis_model_init_rpackets(const artis_model *m, int nts, int npkts, uint64_t seed, double etot,
                              artis_packet *out);

int64_t artis_model_npts_model(const artis_model *m);
/* RADFIELDBINCOUNT of the nebular options, 0 otherwise */
int artis_model_radfield_nbins(const artis_model *m);
int artis_model_total_nlte_levels(const artis_model *m);
const int32_t *artis_model_ion_ionstage(const artis_model *m);
void artis_model_ion_ground_statweight(const artis_model *m, float *out);  /* [nions_total] g of each ground level */
/* the configuration the model was built with (after artis_model_from_files adopted input.txt's values) */
void artis_model_config(const artis_model *m, artis_synth_config *out);

/* Gamma-ray line spectrum of stand-in nuclide `nuc` (energies in MeV, photons per decay), as read by
 * read_gamma_spectrum (gammapkt.cc:58-89); nucdecayenergygamma = sum E p.  Nuclides (decay.cc stand-in):
 * 0 Ni56 (EC), 1 Co56 (EC / beta+), 2 Fe52-like (gamma energy but no line list -> k-packet,
 * gammapkt.cc:266-270), 3 a beta- emitter, 4 an alpha emitter (no gammas). */
int artis_model_set_gamma_lines(artis_model *m, int nuc, int nlines, const double *energy_mev, const double *prob);
const artis_gamma_spectra *artis_model_gamma_spectra(const artis_model *m);

/* Initial radioactive pellets (packet_init + place_pellet + setup_radioactive_pellet, packet.cc:18-149,
 * decay.cc:1371-1458): cell ~ rho * q, position uniform in the cell at tmin, decay path by energy share,
 * tdecay by the chain's summed exponential draws in (t_model, tmax) (decay.cc:716-732), a fraction
 * frac_initial of USE_MODEL_INITIAL_ENERGY pellets with tdecay = tmin. */
int artis_model_init_pellets(const artis_model *m, int npkts, uint64_t seed, double etot, double t_model_days,
                             double frac_initial, artis_packet *out);

#ifdef __cplusplus
}
#endif
#endif
