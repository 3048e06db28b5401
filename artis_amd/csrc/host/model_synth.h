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
} artis_synth_config;

typedef struct artis_model artis_model;

void artis_synth_default_config(artis_synth_config *cfg);
artis_model *artis_model_synth(const artis_synth_config *cfg);
void artis_model_free(artis_model *m);

const artis_atomic_tables *artis_model_atomic(const artis_model *m);
const artis_geometry *artis_model_geometry(const artis_model *m);
const artis_cell_state *artis_model_cellstate(const artis_model *m);
void artis_model_run_params(const artis_model *m, artis_run_params *out);

/* LTE update_grid stand-in for timestep nts (densities scaled to ts_mid[nts]). */
int artis_model_set_timestep(artis_model *m, int nts);

/* Initial r-packets at the start of timestep nts: cell ~ rho*vol, isotropic direction, nu_cmf ~ Planck(T_e)
 * within [NU_MIN_R, NU_MAX_R], equal e_cmf (SURVEY.md §8(d) "pure r-packet benchmark"). */
int artis_model_init_rpackets(const artis_model *m, int nts, int npkts, uint64_t seed, double etot,
                              artis_packet *out);

int64_t artis_model_npts_model(const artis_model *m);

#ifdef __cplusplus
}
#endif
#endif
