/*
 * artis_gpu.h -- C-ABI drop-in boundary of the MI355X packet-propagation engine.
 *
 * Replaces the reference call
 *     void update_packets(const int my_rank, int nts, struct packet *packets);
 * (reference update_packets.h:6, called once per timestep by do_timestep at sn3d.cc:574,
 *  after zero_estimators() sn3d.cc:568 and before mpi_reduce_estimators sn3d.cc:582)
 * with three calls:
 *     artis_gpu_init()              -- once per run: atomic tables + geometry (reference input(), grid_init())
 *     artis_gpu_upload_cellstate()  -- once per timestep after update_grid (reference update_grid.cc:1270)
 *     artis_gpu_update_packets()    -- the hot path (reference update_packets.cc:234-333)
 *
 * Everything crossing this boundary is plain C: pointers, sizes, ints and doubles.  No torch, no HIP types.
 * The packet record is the reference's 304-byte `struct packet` (packet.h:28-73), bit-identical, so the raw
 * `packets_RRRR_tsN.tmp` restart files (sn3d.cc:387-398, packet.cc:198-209) stay valid.
 *
 * All returns: 0 on success, negative artis_status on failure.  The C++ host mirror
 * (artis_amd/csrc/host/update_packets_gpu.cc) turns a failure into the reference's abort()
 * (assert_always, sn3d.h:17-29).
 */
#ifndef ARTIS_GPU_H
#define ARTIS_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------------------------------------------------ */
/* Packet record: reference packet.h:6-73 (types), boundary.h:4-12 (last_cross). sizeof == 304, offsets checked   */
/* by static asserts in artis_layout_check.h and by tests/test_abi.py.                                          */
/* ------------------------------------------------------------------------------------------------------------ */
enum artis_packet_type {
  ARTIS_TYPE_ESCAPE = 32,
  ARTIS_TYPE_RADIOACTIVE_PELLET = 100,
  ARTIS_TYPE_GAMMA = 10,
  ARTIS_TYPE_RPKT = 11,
  ARTIS_TYPE_KPKT = 12,
  ARTIS_TYPE_MA = 13,
  ARTIS_TYPE_NTLEPTON = 20,
  ARTIS_TYPE_NONTHERMAL_PREDEPOSIT = 21,
  ARTIS_TYPE_PRE_KPKT = 120,
  ARTIS_TYPE_GAMMA_KPKT = 121,
};

enum artis_cell_boundary {
  ARTIS_NEG_X = 101,
  ARTIS_POS_X = 102,
  ARTIS_NEG_Y = 103,
  ARTIS_POS_Y = 104,
  ARTIS_NEG_Z = 105,
  ARTIS_POS_Z = 106,
  ARTIS_NONE = 107,
};

typedef struct artis_mastate {
  int32_t element;
  int32_t ion;
  int32_t level;
  int32_t activatingline;
} artis_mastate;

typedef struct artis_packet {
  int32_t where;             /*   0 */
  int32_t type;              /*   4  enum artis_packet_type */
  int32_t last_cross;        /*   8  enum artis_cell_boundary */
  int32_t interactions;      /*  12 */
  int32_t nscatterings;      /*  16 */
  int32_t last_event;        /*  20 */
  double pos[3];             /*  24 */
  double dir[3];             /*  48 */
  double e_cmf;              /*  72 */
  double e_rf;               /*  80 */
  double nu_cmf;             /*  88 */
  double nu_rf;              /*  96 */
  int32_t next_trans;        /* 104 */
  int32_t emissiontype;      /* 108 */
  double em_pos[3];          /* 112 */
  int32_t em_time;           /* 136 */
  int32_t _pad0;             /* 140 */
  double prop_time;          /* 144 */
  int32_t absorptiontype;    /* 152 */
  int32_t trueemissiontype;  /* 156 */
  int32_t trueem_time;       /* 160 */
  int32_t _pad1;             /* 164 */
  double absorptionfreq;     /* 168 */
  double absorptiondir[3];   /* 176 */
  double stokes[3];          /* 200 */
  double pol_dir[3];         /* 224 */
  double tdecay;             /* 248 */
  int32_t escape_type;       /* 256 */
  int32_t escape_time;       /* 260 */
  int32_t scat_count;        /* 264 */
  int32_t number;            /* 268 */
  uint8_t originated_from_particlenotgamma; /* 272  (C++ bool in the reference) */
  uint8_t _pad2[3];          /* 273 */
  int32_t pellet_decaytype;  /* 276 */
  int32_t pellet_nucindex;   /* 280 */
  float trueemissionvelocity;/* 284 */
  artis_mastate mastate;     /* 288 */
} artis_packet;              /* 304 */

/* ------------------------------------------------------------------------------------------------------------ */
/* Atomic data (read-only for the whole run).  Flattened form of the reference globals::elements / linelist /    */
/* allcont / groundcont / LUTs (globals.h:44-160, 273-294; input.cc:747-1186, 1439-1652).                       */
/* Index conventions follow the reference: ions are numbered globally by get_uniqueionindex (atomic.cc:246),   */
/* levels by get_uniquelevelindex (atomic.cc:278); `level` fields inside per-ion records are ion-local.          */
/* ------------------------------------------------------------------------------------------------------------ */
typedef struct artis_atomic_tables {
  int32_t nelements;
  int32_t maxnions;          /* get_max_nions() */
  int32_t nions_total;       /* get_includedions() */
  int32_t nlevels_total;
  int32_t nlines;
  int32_t nbfcontinua;
  int32_t nbfcontinua_ground;
  int32_t ncoolingterms;
  int32_t nphixspoints;              /* globals::NPHIXSPOINTS */
  double nphixsnuincrement;          /* globals::NPHIXSNUINCREMENT */
  double last_phixs_nuovernuedge;    /* atomic.cc:8 */
  int32_t phixs_file_version;        /* 1 or 2 (atomic.cc:12) */
  int32_t tablesize;                 /* TABLESIZE */
  double mintemp, maxtemp;           /* MINTEMP, MAXTEMP; T_step_log derived as ratecoeff.cc:1004 */

  /* elements [nelements] */
  const int32_t *elem_anumber;
  const int32_t *elem_nions;
  const int32_t *elem_uniqueionoffset; /* unique ion index of ion 0 */

  /* ions [nions_total] */
  const int32_t *ion_ionstage;
  const int32_t *ion_nlevels;
  const int32_t *ion_uniqueleveloffset; /* unique level index of level 0 */
  const int32_t *ion_ionisinglevels;
  const int32_t *ion_maxrecombininglevel;
  const int32_t *ion_coolingoffset;
  const int32_t *ion_ncoolingterms;
  const double *ion_ionpot;

  /* levels [nlevels_total] */
  const double *level_epsilon;
  const float *level_stat_weight;
  const int32_t *level_nuptrans;
  const int32_t *level_uptrans_offset;     /* into uptrans_lineindex */
  const int32_t *level_ndowntrans;
  const int32_t *level_downtrans_offset;   /* into downtrans_lineindex */
  const int32_t *level_nphixstargets;      /* raw count; get_nphixstargets() applies the ionising-level rule */
  const int32_t *level_phixstargets_offset;/* into phixstarget_* */
  const int32_t *level_cont_index;         /* reference levellist_entry::cont_index (negative) */
  const int32_t *level_closestgroundlevelcont; /* element*maxnions+ion, or -1 */
  const int32_t *level_phixstable;         /* row into phixs_xs, -1 if none */
  const int32_t *uptrans_lineindex;
  const int32_t *downtrans_lineindex;
  const int32_t *phixstarget_levelindex;   /* ion-local level index in ion+1 */
  const double *phixstarget_probability;
  const float *phixs_xs;                   /* [ntables * nphixspoints], cm^2 */

  /* lines [nlines], sorted by descending nu (reference linelist_entry, globals.h:133-144) */
  const double *line_nu;
  const float *line_einstein_A;
  const float *line_osc_strength;
  const float *line_coll_str;
  const int32_t *line_elementindex;
  const int32_t *line_ionindex;
  const int32_t *line_upperlevelindex;
  const int32_t *line_lowerlevelindex;
  const uint8_t *line_forbidden;

  /* all bf continua [nbfcontinua], sorted by ascending nu_edge (reference fullphixslist, globals.h:53-63) */
  const double *allcont_nu_edge;
  const int32_t *allcont_element;
  const int32_t *allcont_ion;
  const int32_t *allcont_level;
  const int32_t *allcont_phixstargetindex;
  const int32_t *allcont_upperlevel;
  const int32_t *allcont_phixstable;
  const double *allcont_probability;
  const int32_t *allcont_index_in_groundphixslist;

  /* ground-level continua [nbfcontinua_ground], ascending nu_edge (reference groundphixslist, globals.h:65-71) */
  const double *groundcont_nu_edge;
  const int32_t *groundcont_element;
  const int32_t *groundcont_ion;
  const int32_t *groundcont_level;
  const int32_t *groundcont_phixstargetindex;

  /* rate-coefficient LUTs [tablesize * nbfcontinua], indexed get_bflutindex (sn3d.h:64-69) */
  const double *spontrecombcoeff;
  const double *corrphotoioncoeff;
  const double *bfcooling_coeff;

  /* k-packet cooling list [ncoolingterms] (kpkt.cc:339-426) */
  const int32_t *coolinglist_type;      /* 880 ff, 881 fb, 882 collexc, 883 collion */
  const int32_t *coolinglist_element;
  const int32_t *coolinglist_ion;
  const int32_t *coolinglist_level;
  const int32_t *coolinglist_upperlevel;

  /* ABI 6 -- NLTE populations (NLTE_POPS_ON; ltepop.cc:349-415, input.cc:1711-1746): per ion the number of NLTE
     excited levels (levels 1..nlevels_nlte; the remaining excited levels form one superlevel if there are any) and
     the index of its first entry in a cell's nlte_pops vector; total_nlte_levels entries per cell.  NULL / 0 when
     NLTE populations are off. */
  const int32_t *ion_nlevels_nlte;
  const int32_t *ion_first_nlte;
  int32_t total_nlte_levels;
  /* binned radiation field (MULTIBIN_RADFIELD_MODEL_ON; radfield.cc:131-188, 574-608): upper frequency edge of each
     bin and the lower edge of bin 0 */
  int32_t radfield_nbins;
  const double *radfield_nu_upper;   /* [radfield_nbins] */
  double radfield_nu_lower_first;
} artis_atomic_tables;

/* ------------------------------------------------------------------------------------------------------------ */
/* Geometry + time grid (reference grid.h:20-65, grid.cc:2028-2102, input.cc:2226-2381).                       */
/* ------------------------------------------------------------------------------------------------------------ */
enum artis_grid_type { ARTIS_GRID_UNIFORM = 1, ARTIS_GRID_SPHERICAL1D = 2 };

typedef struct artis_geometry {
  int32_t grid_type;
  int32_t ncoordgrid[3];
  int32_t ngrid;
  int32_t npts_model;          /* empty propagation cells map to mgi == npts_model */
  const double *cell_pos_min;  /* [ngrid * 3] at tmin (grid::cell[].pos_min) */
  const int32_t *cell_mgi;     /* [ngrid] */
  const double *modelcell_wid_init; /* [npts_model] radial extent at tmin (spherical only; may be NULL) */
  double coordmax[3];
  double tmin, tmax, rmax, vmax;
  int32_t ntstep;
  const double *ts_start;      /* [ntstep] */
  const double *ts_width;
  const double *ts_mid;
  double nu_min_r, nu_max_r;   /* NU_MIN_R, NU_MAX_R (sample_planck range) */
} artis_geometry;

/* ------------------------------------------------------------------------------------------------------------ */
/* Per-timestep model-cell state written by the host update_grid (reference modelgrid_t, grid.h:33-65).        */
/* All arrays are indexed by model-grid index mgi in [0, npts_model).                                          */
/* ------------------------------------------------------------------------------------------------------------ */
typedef struct artis_cell_state {
  const float *Te, *TR, *TJ, *W, *nne, *nnetot, *rho, *kappagrey;
  const int16_t *thick;
  const float *elem_abundance;        /* [npts_model * nelements] mass fractions */
  const float *groundlevelpop;        /* [npts_model * nions_total] */
  const float *partfunct;             /* [npts_model * nions_total] */
  const double *totalcooling;         /* [npts_model] */
  const double *cooling_contrib_ion;  /* [npts_model * nions_total] */
  const double *corrphotoionrenorm;   /* [npts_model * nelements * maxnions] */
  const float *ffegrp;                /* [npts_model] Fe-group mass fraction (grid.cc:223), gamma opacities;
                                         may be NULL when no gamma packets are propagated */
  /* ABI 6 (all may be NULL when the option that reads them is off) */
  const double *nlte_pops;            /* [npts_model * total_nlte_levels] NLTE level population / rho (grid.h:33-65);
                                         < -0.9: no solution yet, LTE is used (ltepop.cc:367-370) */
  const float *radfield_bin_TR;       /* [npts_model * radfield_nbins] radfieldbin_solutions T_R and W of the fitted */
  const float *radfield_bin_W;        /*   dilute blackbody per bin (radfield.cc:908-920); W < 0: no fit */
  const float *bfrate_estimator;      /* [npts_model * nbfcontinua] prev_bfrate_normed, the normalised bf-rate
                                         estimators of the previous timestep (radfield.cc:73, 1306-1316, used by
                                         get_corrphotoioncoeff, ratecoeff.cc:1255-1261); <= 0: none */
  const double *nt_deposition_rate_density;  /* [npts_model] (nonthermal.cc:659) */
  const double *nt_ionization_ratecoeff;     /* [npts_model * nions_total] nt_ionization_ratecoeff (nonthermal.cc:
                                                1684-1709, evaluated by the host update_grid incl. its fallbacks) */
  const float *nt_prob_num_auger;            /* [npts_model * nions_total * (nt_max_auger_electrons + 1)] */
  const float *nt_ionenfrac_num_auger;       /*   nt_solution prob_num_auger / ionenfrac_num_auger (nonthermal.cc:136-139) */
} artis_cell_state;

/* Run-time switches of input.txt / artisoptions.h that change hot-path behaviour. */
typedef struct artis_run_params {
  uint32_t seed;               /* input.txt line 1 (pre_zseed) */
  int32_t rank;                /* this rank's packet ensemble ("rank" of the reference MPI run) */
  int32_t opacity_case;        /* input.txt: 4 = full opacity */
  int32_t do_r_lc;             /* input.txt r-light-curve flag (derived as input.cc:1976-1979) */
  int32_t do_rlc_est;          /* input.txt line 9 */
  int32_t n_kpktdiffusion_timesteps;
  float kpktdiffusion_timescale;
  double max_path_step;        /* globals::max_path_step (update_grid.cc:1400) */
  int32_t pol_dipole;          /* DIPOLE: 1 = dipole rejection scattering (polarization.cc:26-53) */
  int32_t relativistic_doppler;/* USE_RELATIVISTIC_DOPPLER_SHIFT */
  int32_t record_linestat;     /* RECORD_LINESTAT */
  double gamma_grey;           /* input.txt "use grey opacity for gammas?" (input.cc:1992); < 0: full treatment */
  int32_t instant_particle_deposition; /* INSTANT_PARTICLE_DEPOSITION (update_packets.cc:23) */
  int32_t nt_solve_spencerfano;/* NT_ON && NT_SOLVE_SPENCERFANO (nonthermal.cc:1883): not propagated here */
  int32_t excitation_temperature; /* LTEPOP_EXCITATIONTEMPERATURE of calculate_levelpop_lte (ltepop.cc:338):
                                     ARTIS_TEXC_TJ (artisoptions_classic.h:32) or ARTIS_TEXC_TE
                                     (artisoptions_kilonova_lte.h:36, artisoptions_nltenebular.h:36) */
  /* ABI 6: the nebular options (artisoptions_nltenebular.h) */
  int32_t nlte_pops_on;                 /* NLTE_POPS_ON */
  int32_t multibin_radfield;            /* MULTIBIN_RADFIELD_MODEL_ON: bin estimators; J_nu from the bins ... */
  int32_t first_nlte_radfield_timestep; /* ... from timestep FIRST_NLTE_RADFIELD_TIMESTEP on (radfield.cc:901) */
  int32_t detailed_bf_estimators;       /* DETAILED_BF_ESTIMATORS_ON: bfrate_raw, kappa_bf inclusion (rpkt.cc:1116) */
  int32_t detailed_bf_usefromtimestep;  /* DETAILED_BF_ESTIMATORS_USEFROMTIMESTEP (ratecoeff.cc:1262) */
  int32_t no_lut_photoion;              /* NO_LUT_PHOTOION: corrphotoioncoeff by integration (ratecoeff.cc:1184-1245) */
  int32_t no_lut_bfheating;             /* NO_LUT_BFHEATING: no bfheatingestimator (rpkt.cc:576-613) */
  int32_t nt_on;                        /* NT_ON: non-thermal ionisation macro-atom action (macroatom.cc:143-146) */
  int32_t nt_max_auger_electrons;       /* NT_MAX_AUGER_ELECTRONS (artisoptions_nltenebular.h:193) */
  double minpop;                        /* MINPOP: 1e-30 classic (artisoptions_classic.h:78), 1e-40 kilonova and
                                           nebular (artisoptions_kilonova_lte.h:79, artisoptions_nltenebular.h:82);
                                           0 is read as 1e-30 */
  /* ABI 10: the Compton / pair-production emissivity estimators of gamma packets (compton_emiss_cont /
     pp_emiss_cont, emissivities.cc:14-136, called from do_gamma, gammapkt.cc:619-657).  The reference sets
     do_comp_est = do_r_lc ? false : estim_switch(nts) every timestep (sn3d.cc:539); the engine evaluates the same
     rule per timestep when comp_est is 1 (0: never, for callers that do not ask for compton_emiss). */
  int32_t comp_est;
  int32_t emiss_offset;                 /* globals::emiss_offset = get_nul(nusyn_min) (input.cc:1813-1818) */
  int32_t emiss_max;                    /* globals::emiss_max <= ARTIS_EMISS_MAX */
  int32_t _pad_comp;
  double time_syn_first, time_syn_last; /* time_syn[0], time_syn[nsyn_time - 1] of estim_switch
                                           (emissivities.cc:250-257) */
  double syn_dir[3];                    /* globals::syn_dir (the observer direction of compton_emiss_cont) */
} artis_run_params;
enum artis_excitation_temperature { ARTIS_TEXC_TJ = 0, ARTIS_TEXC_TE = 1 };

/* ------------------------------------------------------------------------------------------------------------ */
/* Accumulators (reference radfield J/nuJ, globals::*estimator, time_step[nts].*, ecounter/acounter, stats).  */
/* Un-normalised sums with the reference index conventions; the engine ADDS into them (zero_estimators is     */
/* the caller's job, emissivities.cc:138).                                                                     */
/* ------------------------------------------------------------------------------------------------------------ */
#define ARTIS_COUNTER_COUNT 34   /* stats.h:49-83 */

typedef struct artis_estimators {
  double *J;                   /* [npts_model]  radfield.cc:100 */
  double *nuJ;                 /* [npts_model]  radfield.cc:108 */
  double *ffheatingestimator;  /* [npts_model] */
  double *colheatingestimator; /* [npts_model] */
  double *gammaestimator;      /* [npts_model * nelements * maxnions]  rpkt.cc:596 */
  double *bfheatingestimator;  /* [npts_model * nelements * maxnions] */
  int32_t *ecounter;           /* [nlines]  RECORD_LINESTAT (may be NULL) */
  int32_t *acounter;           /* [nlines] */
  double cmf_lum, gamma_dep, positron_dep, electron_dep, electron_emission, alpha_dep, alpha_emission,
      gamma_emission;          /* time_step[nts].* (globals.h:20-40) */
  int64_t pellet_decays;
  int64_t nesc;                /* globals::nesc */
  int64_t counters[ARTIS_COUNTER_COUNT];
  double *rpkt_emiss;          /* [npts_model] grey gamma heating estimator rlc_emiss_gamma (grey_emissivities.cc:28-77,
                                  globals.cc:30); may be NULL */
  double nt_energy_deposited;  /* nonthermal.cc:115, added by do_ntlepton (nonthermal.cc:1878) */
  /* ABI 6 (may be NULL when the option is off) */
  double *bfrate_raw;          /* [npts_model * nbfcontinua] DETAILED_BF_ESTIMATORS_ON (radfield.cc:764-829) */
  double *radfield_J_raw;      /* [npts_model * radfield_nbins] MULTIBIN_RADFIELD_MODEL_ON (radfield.cc:859-866) */
  double *radfield_nuJ_raw;
  int64_t *radfield_contribcount;
  /* ABI 10 (may be NULL unless artis_run_params.comp_est is 1) */
  float *compton_emiss;        /* [(npts_model + 1) * ARTIS_EMISS_MAX] globals::compton_emiss (grid.cc:1699), float as
                                  the reference; the engine sums in double and adds its sum once */
} artis_estimators;
#define ARTIS_EMISS_MAX 2      /* EMISS_MAX (globals.h:223) */

/* ------------------------------------------------------------------------------------------------------------ */
/* Gamma-ray line spectra per nuclide, as read by read_gamma_spectrum (gammapkt.cc:58-89) into gamma_spectra    */
/* (gammapkt.cc:27-33), plus nucdecayenergygamma(z, a) (decay.cc) that choose_gamma_ray divides by             */
/* (gammapkt.cc:234).  Indexed by the reference nuclide index = packet.pellet_nucindex.                        */
/* ------------------------------------------------------------------------------------------------------------ */
typedef struct artis_gamma_spectra {
  int32_t nnuclides;
  const int32_t *nuc_nlines;        /* [nnuclides]; 0: no gamma spectrum, the pellet becomes a k-packet */
  const int32_t *nuc_line_offset;   /* [nnuclides] into line_energy / line_probability */
  const double *nuc_endecay_gamma;  /* [nnuclides] average gamma energy per decay [erg] */
  const double *line_energy;        /* [sum nlines] erg */
  const double *line_probability;   /* [sum nlines] photons per decay */
} artis_gamma_spectra;

/* ------------------------------------------------------------------------------------------------------------ */
/* Virtual packets (VPKT_ON): vpkt.cc.  Every r-packet emission -- electron scattering (rpkt.cc:358-363),        */
/* macro-atom bb / fb deactivation (macroatom.cc:292-295, 376-379), k-packet ff / fb cooling (kpkt.cc:631-634,  */
/* 691-694) -- spawns one virtual packet per observer direction and frequency range (vpkt_call_estimators,     */
/* vpkt.cc:837-896), traced to the grid edge through line and continuum opacity without interacting            */
/* (rlc_emiss_vpkt, vpkt.cc:76-368) and binned with weight p_n e^-tau into the polarised spectra vstokes_i/q/u  */
/* (add_to_vspecpol, vpkt.cc:388-406) and, optionally, the velocity-grid map (add_to_vpkt_grid, vpkt.cc:581-627).*/
/* The parameters are those of vpkt.txt (read_parameterfile_vpkt, vpkt.cc:667-835) plus the compile-time       */
/* binning constants of vpkt.h:30-47, given here at run time.                                                  */
/* ------------------------------------------------------------------------------------------------------------ */
#define ARTIS_VPKT_MAX_SPECTRA 8   /* Nspectra (opacity choices per observer) */
#define ARTIS_VPKT_MRANGE 4        /* frequency ranges (MRANGE = 1 in vpkt.h:47) */
#define ARTIS_VPKT_MRANGE_GRID 5   /* MRANGE_GRID (vpkt.h:30) */

typedef struct artis_vpkt_params {
  int32_t nobs;                    /* Nobs */
  const double *nz_obs;            /* [nobs] cos(theta), after the +-1 -> +-0.9999 rewrite (vpkt.cc:680-687) */
  const double *phi_obs;           /* [nobs] radians */
  int32_t nspectra;                /* Nspectra <= ARTIS_VPKT_MAX_SPECTRA */
  const double *exclude;           /* [nspectra] 0: all opacity; -1: no lines; -2: no bf; -3: no ff; -4: no es;
                                      Z > 0: without the lines of element Z (vpkt.cc:209-218, 272-277) */
  double tmin_vspec, tmax_vspec;   /* vpkt.h:42-43 (10 d, 30 d) */
  double numin_vspec, numax_vspec; /* vpkt.h:36-37 */
  int32_t vmtbins, vmnubins;       /* VMTBINS (30), VMNUBINS (2500) */
  double tmin_vspec_input, tmax_vspec_input;  /* vpkt.txt time window (within [tmin_vspec, tmax_vspec]) */
  int32_t nrange;                  /* Nrange <= ARTIS_VPKT_MRANGE */
  double numin_vspec_input[ARTIS_VPKT_MRANGE], numax_vspec_input[ARTIS_VPKT_MRANGE];
  double tau_max_vpkt;
  int32_t vgrid_flag;              /* 1: velocity-grid map */
  double tmin_grid, tmax_grid;
  int32_t nrange_grid;             /* <= ARTIS_VPKT_MRANGE_GRID */
  double nu_grid_min[ARTIS_VPKT_MRANGE_GRID], nu_grid_max[ARTIS_VPKT_MRANGE_GRID];
  int32_t ny_vgrid, nz_vgrid;      /* NY_VGRID, NZ_VGRID (50, 50; vpkt.h:31-32) */
  int32_t nprocs;                  /* globals::nprocs of the add_to_vspecpol normalisation (vpkt.cc:398-399) */
  int64_t spawn_capacity;          /* engine only: virtual-packet spawn records held in HBM per event round;
                                      0 = default (16 per packet, at least 2^20) */
} artis_vpkt_params;

/* Accumulators of the virtual packets, un-normalised beyond what add_to_vspecpol / add_to_vpkt_grid apply.
 * vstokes_* [vmtbins][nobs * nspectra][vmnubins] (vstokes_i[nt][ind_comb].flux[nnu], vpkt.cc:21-23, 391);
 * vgrid_* [ny_vgrid][nz_vgrid][nrange_grid][nobs] (vgrid_i[n][m].flux[range][obs], vpkt.cc:53-55), may be NULL
 * when vgrid_flag == 0; the counters are nvpkt / nvpkt_esc1-3 (vpkt.cc:69-74). */
typedef struct artis_vpkt_result {
  double *vstokes_i, *vstokes_q, *vstokes_u;
  double *vgrid_i, *vgrid_q, *vgrid_u;
  int64_t nvpkt, nvpkt_esc1, nvpkt_esc2, nvpkt_esc3;
} artis_vpkt_result;

enum artis_status {
  ARTIS_OK = 0,
  ARTIS_ERR_NOT_INITIALISED = -1,
  ARTIS_ERR_HIP = -2,
  ARTIS_ERR_BAD_ARGUMENT = -3,
  ARTIS_ERR_NO_CELLSTATE = -4,
  ARTIS_ERR_PACKET_FAULT = -5,   /* a packet hit an abort() path of the reference (see artis_gpu_last_error) */
  ARTIS_ERR_UNSUPPORTED = -6,    /* a packet type / option this build does not propagate */
};

/* --- lifecycle ------------------------------------------------------------------------------------------- */
/* Bind the engine to HIP device `device` and upload read-only tables.  Replaces the table setup done by
 * input(rank) (input.cc:1754) and grid_init (grid.cc:2132) as seen by update_packets. */
int artis_gpu_init(int device, const artis_atomic_tables *atomic, const artis_geometry *geom,
                   const artis_run_params *params);
void artis_gpu_finalize(void);
/* Upload the gamma-ray line spectra used by pellet decays (replaces gammapkt::init_gamma_linelist,
 * gammapkt.cc:194, as seen by pellet_gamma_decay / do_gamma).  Needed before pellets or gamma packets are
 * propagated; without it such packets fail with ARTIS_ERR_UNSUPPORTED. */
int artis_gpu_init_gamma(const artis_gamma_spectra *spectra);

/* Upload the per-cell state produced by update_grid for timestep nts and build the engine's per-cell tables
 * (level populations, cumulative k-packet cooling lists) that replace the per-thread cellhistory
 * (update_grid.cc:659-761). */
int artis_gpu_upload_cellstate(int nts, const artis_cell_state *cells);

/* The drop-in for update_packets(my_rank, nts, packets): packets are copied to HBM, propagated to the end of
 * timestep nts, copied back IN PLACE (same order as given), and estimator sums are ADDED into *est. */
int artis_gpu_update_packets(int my_rank, int nts, artis_packet *packets, int npkts, artis_estimators *est);

/* --- device-resident path (bench / multi-timestep runs without PCIe traffic) ----------------------------- */
int artis_gpu_packets_upload(const artis_packet *packets, int npkts);   /* host AoS -> HBM SoA */
int artis_gpu_packets_download(artis_packet *packets, int npkts);       /* HBM SoA -> host AoS */
int artis_gpu_packets_snapshot(void);          /* keep a device copy of the current packets */
int artis_gpu_packets_restore(void);           /* reset packets to the snapshot (device-to-device) */
int artis_gpu_update_packets_resident(int my_rank, int nts);            /* propagate resident packets */
int artis_gpu_estimators_zero(void);                                    /* zero the device accumulators */
int artis_gpu_estimators_download(artis_estimators *est);               /* ADD device sums into *est */
/* Packed device estimator block (doubles then int64 counters) for an RCCL all-reduce done by the caller:
 * copy to / from a caller-owned device buffer of 8 * artis_gpu_estimator_block_doubles bytes. */
size_t artis_gpu_estimator_block_doubles(void);
int artis_gpu_estimator_block_to_device(void *dst_device);
int artis_gpu_estimator_block_from_device(const void *src_device);
/* The same block layout on the host (no device needed), so a host-side reduction (MPI / gloo) of
 * artis_estimators sums exactly what the device block carries:
 *   [J | nuJ | ffheating | colheating | rpkt_emiss (npts_model each) | gammaestimator | bfheatingestimator
 *    (npts_model * nelements * maxnions each) | cmf_lum gamma_dep positron_dep electron_dep electron_emission
 *    alpha_dep alpha_emission gamma_emission nt_energy_deposited pellet_decays | bfrate_raw (npts_model * nbf_est)
 *   | radfield_J_raw | radfield_nuJ_raw | radfield_contribcount (npts_model * nbins_est each)
 *   | compton_emiss ((npts_model + 1) * ARTIS_EMISS_MAX, as float64; ABI 10) | ecounter | acounter
 *    (nlines each) | counters (ARTIS_COUNTER_COUNT) | nesc]   -- counts as float64 (exact below 2^53).
 * nbf_est = nbfcontinua under DETAILED_BF_ESTIMATORS_ON, else 0; nbins_est = radfield_nbins under
 * MULTIBIN_RADFIELD_MODEL_ON, else 0 (the engine's block has the sections its run parameters switch on).
 * pack: NULL array pointers of *est pack as zeros; unpack OVERWRITES *est (NULL arrays skipped). */
size_t artis_estimator_block_len(int npts_model, int nelements, int maxnions, int nlines, int nbf_est, int nbins_est);
int artis_estimator_block_pack(const artis_estimators *est, int npts_model, int nelements, int maxnions, int nlines,
                               int nbf_est, int nbins_est, double *block);
int artis_estimator_block_unpack(const double *block, int npts_model, int nelements, int maxnions, int nlines,
                                 int nbf_est, int nbins_est, artis_estimators *est);
/* After a host-side SUM of the blocks of nranks ranks: divide the eight time_step scalars (cmf_lum .. gamma_emission)
 * by nranks, as mpi_reduce_estimators does after its MPI_Allreduce (sn3d.cc:370-377).  artis_gpu_estimators_allreduce
 * applies the same division to the device block. */
int artis_estimator_block_average_scalars(double *block, int npts_model, int nelements, int maxnions, int nranks);

/* --- multi-GPU: RCCL over xGMI (the reference's mpi_reduce_estimators, sn3d.cc:316-377, radfield.cc:1502-1564) */
/* One process per GPU; every rank propagates its own full-energy ensemble and the only exchange per timestep
 * is the SUM of the packed device estimator block.  Rank 0 creates the id (ncclGetUniqueId), the host hands
 * it to every rank (MPI_Bcast in sn3d, a torch.distributed broadcast in bench.py), each rank joins with
 * artis_gpu_comm_init on the engine's device; artis_gpu_estimators_allreduce then all-reduces the block in
 * HBM on the engine stream (ncclAllReduce, ncclSum, ncclFloat64).  id: ARTIS_COMM_ID_BYTES opaque bytes. */
#define ARTIS_COMM_ID_BYTES 128
int artis_gpu_comm_unique_id(void *id);
int artis_gpu_comm_init(int rank, int nranks, const void *id);
int artis_gpu_estimators_allreduce(void);
void artis_gpu_comm_finalize(void);

/* --- timing / introspection --------------------------------------------------------------------------------- */
/* Milliseconds of the transport kernel(s) of the last update_packets call, measured with HIP events on the
 * engine's own stream (the stream the kernels run on). */
double artis_gpu_last_transport_ms(void);
/* Milliseconds of the per-cell precompute kernels of the last artis_gpu_upload_cellstate (HIP events). */
double artis_gpu_last_precompute_ms(void);
/* Per-call event counts from the device (steps, lines scanned, kappa evaluations, ...), for the byte model. */
#define ARTIS_WORK_COUNT 16
int artis_gpu_last_work_counts(int64_t out[ARTIS_WORK_COUNT]);
/* Coverage of the per-cell tables the engine sized at init (ABI 9, 11): out[0] non-empty cells; out[1] cells with
 * a row of line coefficients (numbered centre outwards; the rest gather populations in the line walk) and out[2]
 * their bytes; out[3] cells with a whole row of macro-atom key records (row mode: all of them) and out[4] their
 * bytes.  Level mode (the rows do not fit the budget; ABI 11): records per (cell, level) pair, placed at every
 * artis_gpu_upload_cellstate on the pairs with the most (sampled, decaying) jumps per record line in the past
 * transports (whole cells centre outwards before the first transport); out[5] bytes of the per-pair action totals
 * a jump without a record reads; out[6] / out[7] macro-atom jumps of the last transport made from a record / all
 * its jumps; out[8] records of the current placement, out[9] their bytes, out[10] the pool's bytes.  The split
 * never changes a result. */
#define ARTIS_TABLE_INFO_COUNT 11
int artis_gpu_table_info(int64_t out[ARTIS_TABLE_INFO_COUNT]);
/* Emergent spectrum and light curve of the escaped r-packets among the resident packets, binned on the device:
 * the binning of write_partial_lightcurve_spectra (spectrum.cc:641-721) -- add_to_spec (spectrum.cc:339-362,
 * angle-averaged, no emission-resolved columns) and add_to_lc_res (light_curve.cc:34-54) -- over
 * nnubins log bins in [nu_min_r, nu_max_r] (MNUBINS = 1000 in the reference).  Overwrites the caller's
 * spec_flux[ntstep * nnubins] (timestep-major), lc_lum[ntstep], lc_lumcmf[ntstep]; nprocs is the rank count
 * the reference divides by (globals::nprocs). */
int artis_gpu_spectrum(int nnubins, int nprocs, double *spec_flux, double *lc_lum, double *lc_lumcmf);

/* The full spectra of exspec / write_partial_lightcurve_spectra (exspec.cc, spectrum.cc:306-452,
 * light_curve.cc:34-62) for the resident packets: add_to_spec_res for every escaped r-packet -- the flux, the
 * emission / true-emission spectra resolved by emitting process (bound-bound per ion, bound-free per ion,
 * free-free: proccount = 2 nelements maxnions + 1 columns, columnindex_from_emissiontype, spectrum.cc:306-337),
 * the absorption spectrum by absorbing ion at absorptionfreq (ioncount = nelements maxnions columns), POL_ON
 * Stokes I/Q/U flux and their emission/absorption spectra -- and add_to_lc_res for the r-packet and gamma-ray
 * light curves.  abin -1: all directions; 0 .. ARTIS_MABINS-1: only packets escaping into that direction bin
 * (get_escapedirectionbin about syn_dir, vectors.h:158-193), weighted by ARTIS_MABINS (the gamma-ray light
 * curve is angle-averaged only).  Every array is timestep-major ([ntstep][nnubins][columns]) and ADDED into;
 * NULL arrays are not produced. */
#define ARTIS_MABINS 100
typedef struct artis_spectra_request {
  int32_t nnubins;          /* MNUBINS (1000) log bins over [nu_min_r, nu_max_r] */
  int32_t nprocs;           /* globals::nprocs: every bin is divided by it */
  int32_t abin;
  double syn_dir[3];
} artis_spectra_request;
typedef struct artis_spectra_out {
  double *flux;                       /* [ntstep * nnubins] */
  double *emission, *trueemission;    /* [ntstep * nnubins * proccount] */
  double *absorption;                 /* [ntstep * nnubins * ioncount] */
  double *stokes_flux;                /* [3][ntstep * nnubins]: I, Q, U (POL_ON) */
  double *stokes_emission;            /* [3][ntstep * nnubins * proccount] */
  double *stokes_absorption;          /* [3][ntstep * nnubins * ioncount] */
  double *lc_lum, *lc_lumcmf;         /* [ntstep] */
  double *gamma_lc_lum, *gamma_lc_lumcmf;  /* [ntstep] */
} artis_spectra_out;
int artis_gpu_spectra(const artis_spectra_request *req, artis_spectra_out *out);

/* --- virtual packets (VPKT_ON) ------------------------------------------------------------------------------ */
/* Switch virtual packets on for all following updates (replaces read_parameterfile_vpkt + init_vspecpol +
 * init_vpkt_grid, vpkt.cc:408-443, 547-578, 667-835): allocates and zeroes the device accumulators.  exclude[] > 0
 * refers to the atomic numbers elem_anumber of the tables given to artis_gpu_init.  Emission sites then also set
 * last_cross = NONE before an electron scattering (rpkt.cc:361), as the reference does under VPKT_ON. */
int artis_gpu_vpkt_init(const artis_vpkt_params *params);
int artis_gpu_vpkt_zero(void);                         /* zero the device accumulators and counters */
/* ADD the device accumulators into *out (arrays sized as documented at artis_vpkt_result); the
 * per-timestep counters nvpkt* are zeroed afterwards when reset_counters != 0 (sn3d.cc:621-624). */
int artis_gpu_vpkt_download(artis_vpkt_result *out, int reset_counters);
/* device time (ms) of the virtual-packet kernels of the last update, and the number of spawn records and
 * traced (spawn, observer, range) virtual packets it processed */
int artis_gpu_vpkt_last_stats(double *ms, int64_t *spawns, int64_t *traces);
/* work counters of the last update's virtual packets: [0] cell segments (continuum-opacity evaluations),
 * [1] lines whose opacity was added, [2] active bf continua scanned, [3] virtual packets that escaped */
int artis_gpu_vpkt_last_work(int64_t work[4]);
/* launches of the last update resumed after the spawn buffer filled (ABI 9): the buffer was traced, the spawns
 * that found it full moved to its front, and the r-packet / k-packet launch continued where it stopped */
int64_t artis_gpu_vpkt_last_drains(void);

int64_t artis_gpu_last_rounds(void);  /* event-queue rounds of the last update (0: megakernel path) */
/* device time (ms, HIP events around every launch) and launch count of the last update per kernel class:
 * [0] r-packet (k_rpkt), [1] macro-atom (k_ma), [2] k-packet (k_kpkt), [3] other: classify, gamma, the macro-atom
 * queue binning (k_ma_bin / scan / k_ma_scatter), the exact jumps (k_ma_exact) and the deactivations (k_ma_finish) */
int artis_gpu_last_kernel_times(double ms[4], int64_t launches[4]);
/* the same split finer, ARTIS_KCLASS_COUNT classes: [0] k_rpkt, [1] k_ma, [2] k_kpkt, [3] classify + gamma family
 * (k_classify, k_gamma), [4] queue binning (k_ma_bin(_blk) / scan / k_ma_scatter(_blk), k_r_bin / k_r_scatter),
 * [5] exact jumps (k_ma_exact), [6] deactivations (k_ma_finish); classes 3-6 sum to artis_gpu_last_kernel_times'
 * [3] */
#define ARTIS_KCLASS_COUNT 7
int artis_gpu_last_kernel_class_times(double ms[ARTIS_KCLASS_COUNT], int64_t launches[ARTIS_KCLASS_COUNT]);
const char *artis_gpu_last_error(void);

/* ------------------------------------------------------------------------------------------------------------ */
/* update_grid's temperature / ionisation solution for the LTE-population options (NLTE_POPS_ON false, LUT       */
/* photoionisation and bf heating, NT_ON false: artisoptions_classic.h, artisoptions_kilonova_lte.h), SURVEY.md */
/* §8(f) row 4.  Per model cell, what update_grid_cell does once the estimators are normalised                  */
/* (update_grid.cc:1104-1158, 1199-1205):                                                                       */
/*  - LTE branch (initial_iteration or thick == 1, update_grid.cc:1106-1125): T_e = T_J, precalculate_partfuncts */
/*    (update_grid.cc:23-38), calculate_populations (update_grid.cc:1427-1658);                                 */
/*  - otherwise solve_Te_nltepops (update_grid.cc:763-886): calculate_bfheatingcoeffs (thermalbalance.cc:141-187),*/
/*    precalculate_partfuncts, call_T_e_finder (thermalbalance.cc:397-597: GSL Brent on heating - cooling, each */
/*    evaluation re-solving the ionisation balance with its own Brent on n_e) and calculate_populations;        */
/*  - then kpkt::calculate_cooling_rates (kpkt.cc:84-165): totalcooling and cooling_contrib_ion.               */
/* The run-wide switches (excitation temperature, MINPOP) are those given to artis_gpu_init.                    */
/* ------------------------------------------------------------------------------------------------------------ */
typedef struct artis_te_tables {
  const double *bfheating_coeff;  /* [tablesize * nbfcontinua] globals::bfheating_coeff, get_bflutindex order */
  const float *ion_alpha_sp;      /* [nions_total * tablesize] elements[].ions[].Alpha_sp (input.cc:938) */
} artis_te_tables;

typedef struct artis_te_params {
  double t_current;           /* globals::time_step[nts_for_te].mid (update_grid.cc:804-806) */
  double tmin;                /* globals::tmin */
  double T_min, T_max;        /* MINTEMP, MAXTEMP (the T_e search interval) */
  double accuracy;            /* TEMPERATURE_SOLVER_ACCURACY */
  int32_t initial_iteration;  /* globals::initial_iteration */
  int32_t direct_col_heat;    /* DIRECT_COL_HEAT (artisoptions_kilonova_lte.h:49, artisoptions_nltenebular.h:51): the
                                 collisional heating is the de-excitation sum over every line (thermalbalance.cc:189-216,
                                 223-238) instead of colheatingestimator (ABI 8; was padding, 0 = the classic options) */
} artis_te_params;

#define ARTIS_TE_NRATES 8  /* heatingcoolingrates (thermalbalance.h:4-14): cooling collisional, fb, ff, adiabatic,
                              heating collisional, bf, ff, dep */
typedef struct artis_te_cells {
  int32_t ncells;
  int32_t pad0;
  const int32_t *mgi;                  /* [ncells] model cells to solve */
  /* inputs, indexed by mgi ([npts_model] unless stated) */
  const float *TR, *W, *TJ, *rho;
  const int16_t *thick;                /* before this timestep's update (grid::modelgrid[].thick) */
  const float *elem_abundance;         /* [npts_model * nelements] mass fractions */
  const float *elem_meanweight;        /* [npts_model * nelements] grid::get_element_meanweight [g] */
  const double *vol_init;              /* grid::vol_init_modelcell */
  const double *ffheatingestimator;    /* normalised (update_grid.cc:1133-1134) */
  const double *colheatingestimator;
  const double *gammaestimator;        /* [npts_model * nelements * maxnions] normalised (update_grid.cc:888-975) */
  const double *bfheatingestimator;    /*   ditto */
  const double *heating_dep;           /* do_rlc_est == 3: deposition rate density * nt_frac_heating
                                          (thermalbalance.cc:373-376); NULL: 0 */
  /* in / out */
  float *Te;                           /* in: T_e of the previous timestep; out: the solution */
  float *groundlevelpop;               /* [npts_model * nions_total] in: previous values (partition functions) */
  /* outputs */
  float *nne, *nnetot;
  float *partfunct;                    /* [npts_model * nions_total] */
  double *totalcooling;
  double *cooling_contrib_ion;         /* [npts_model * nions_total] */
  double *heatingcoolingrates;         /* [npts_model * ARTIS_TE_NRATES] of the last thermal-balance evaluation (0 for
                                          LTE-branch cells); may be NULL */
  int32_t *te_iterations;              /* [npts_model] Brent iterations of call_T_e_finder (-1: no root in [T_min,
                                          T_max], 0: LTE branch); may be NULL */
} artis_te_cells;
int artis_gpu_solve_temperatures(const artis_te_tables *tables, const artis_te_params *params, artis_te_cells *cells);
/* The estimator preparation update_grid_cell does before that solution (update_grid.cc:1041-1150, LTE options,
   DO_TITER undefined), for the same cells: estimator_normfactor = 1 / (vol_init tratmid^3) / deltat / nprocs;
   LTE-branch cells: T_J = get_T_J_from_J (radfield.cc:1464-1481), T_R = T_J, W = 1, corrphotoionrenorm = 1;
   other cells: J, nuJ and the ff / collisional heating normalised, update_gamma_corrphotoionrenorm_bfheating_
   estimators (update_grid.cc:888-975: corrphotoionrenorm = Gamma / get_corrphotoioncoeff_ana, then Gamma per
   ground-level population = calculate_iongamma_per_gspop (ratecoeff.cc:1353-1389) with the previous T_R, W, T_e,
   n_e and populations, the bf-heating estimator over get_bfheatingcoeff_ana), then set_params_fullspec
   (radfield.cc:1136-1175) for T_J, T_R, W.  Writes the *_out arrays, which then feed artis_gpu_solve_temperatures
   (cells->TR / W / TJ and the four estimator inputs).  A non-finite corrphotoionrenorm or bf-heating ratio (the
   reference's [fatal] aborts, update_grid.cc:911-918, 959-965) returns ARTIS_ERR_PACKET_FAULT naming the cell and
   leaves the outputs unwritten; so does a GSL abort path of artis_gpu_solve_temperatures. */
typedef struct artis_ug_prepare {
  double deltat;             /* globals::time_step[nts_prev].width (update_grid.cc:1316) */
  double tratmid;            /* globals::time_step[nts].mid / globals::tmin */
  int32_t nprocs;
  int32_t pad0;
  /* raw accumulators of the transport step (summed over ranks) */
  const double *J, *nuJ, *ffheating, *colheating;   /* [npts_model] */
  const double *gammaestimator, *bfheatingestimator; /* [npts_model * nelements * maxnions] */
  const float *nne;          /* previous update_grid state read by calculate_iongamma_per_gspop */
  const float *partfunct;    /* unused (the LUT branch of calculate_iongamma_per_gspop needs no partition function);
                                kept for the layout, may be NULL */
  /* outputs */
  float *TR_out, *W_out, *TJ_out;
  double *ffheating_out, *colheating_out, *gamma_out, *bfheating_out;
  double *corrphotoionrenorm_out;  /* [npts_model * nelements * maxnions] */
} artis_ug_prepare;
int artis_gpu_prepare_temperatures(const artis_te_tables *tables, const artis_te_params *params,
                                   const artis_ug_prepare *prep, const artis_te_cells *cells);

/* device time (ms) of the last artis_gpu_solve_temperatures (the k_te_solve kernel alone) */
double artis_gpu_last_te_ms(void);

/* ------------------------------------------------------------------------------------------------------------ */
/* update_grid for the nebular options (ABI 8; artisoptions_nltenebular.h: NLTE_POPS_ON with                    */
/* NLTE_POPS_ALL_IONS_SIMULTANEOUS, MULTIBIN_RADFIELD_MODEL_ON, DETAILED_BF_ESTIMATORS_ON, NO_LUT_PHOTOION /    */
/* NO_LUT_BFHEATING, NT_ON + NT_SOLVE_SPENCERFANO, DIRECT_COL_HEAT), SURVEY.md §8(f) row 4.  Per listed model     */
/* cell, what update_grid_cell does for timestep nts (update_grid.cc:1012-1205):                                */
/*  - LTE branch (initial_iteration or thick == 1): T_J from J, T_R = T_e = T_J, W = 1, precalculate_partfuncts, */
/*    calculate_populations (LTE phi);                                                                          */
/*  - otherwise: J, nuJ, ff / collisional heating normalised; radfield::fit_parameters (radfield.cc:1136-1291:  */
/*    full-spectrum T_J / T_R / W, and per bin a GSL Brent on the mean frequency of a dilute Planck function with */
/*    GSL qag Planck integrals, the top bin at T_e); normalise_bf_estimators (radfield.cc:1306-1327);           */
/*    solve_Te_nltepops (update_grid.cc:763-886): calculate_bfheatingcoeffs (NO_LUT integrals,                  */
/*    thermalbalance.cc:60-187), then up to NLTEITER + 1 passes of: solve_spencerfano (nonthermal.cc:2522-2713,   */
/*    the SFPTS x SFPTS upper-triangular Spencer-Fano system with its LU refinement, then analyse_sf_solution,  */
/*    nonthermal.cc:1996-2280), call_T_e_finder (thermalbalance.cc:397-597 with calculate_electron_densities),   */
/*    solve_nlte_pops_element for every element (nltepop.cc:798-1113: rate matrix, LTE normalisation, LU solve  */
/*    with iterative refinement), precalculate_partfuncts and calculate_electron_densities, until n_e and T_e    */
/*    change by at most 4 %;                                                                                    */
/*  - then kpkt::calculate_cooling_rates.                                                                      */
/* Third-party arithmetic: GSL's LU (version unpinned; 2.7.1 in the reference CI) is restated as LU with partial */
/* pivoting, right-looking, with column-oriented triangular solves (oracle and engine alike).                  */
/* ------------------------------------------------------------------------------------------------------------ */
#define ARTIS_NT_MAX_AUGER 2  /* NT_MAX_AUGER_ELECTRONS (artisoptions_nltenebular.h:193) */

/* The Spencer-Fano inputs nonthermal::init reads (nonthermal.cc:183-437): impact-ionisation shells of the included
 * ions (collion.txt, Younger fit coefficients) with their g-weighted Auger data (auger-km1993-table2.txt), the
 * binding energies of the work-function approximation (binding_energies.txt), and the energy grid. */
typedef struct artis_nt_shells {
  int32_t nshells;
  int32_t sfpts;                     /* SFPTS (4096) */
  double sf_emin, sf_emax;           /* SF_EMIN, SF_EMAX [eV] (linear grid, SF_USE_LOG_E_INCREMENT false) */
  const int32_t *Z, *nelec, *n, *l;  /* [nshells] in collion.txt order */
  const double *ionpot_ev, *A, *B, *C, *D;
  const double *prob_num_auger;      /* [nshells * (ARTIS_NT_MAX_AUGER + 1)] */
  const float *en_auger_ev;          /* [nshells] */
  const double *electron_binding;    /* [30 * 10] erg, binding_energies.txt */
} artis_nt_shells;

typedef struct artis_nlte_params {
  int32_t nts;                 /* globals::nts_global: the timestep update_grid prepares */
  int32_t num_lte_timesteps;   /* input.txt */
  int32_t initial_iteration;   /* globals::initial_iteration */
  int32_t nprocs;              /* globals::nprocs */
  int32_t nlteiter;            /* NLTEITER (30) */
  int32_t do_rlc_est;          /* 3: gamma-ray heating into the thermal balance (thermalbalance.cc:373-376) */
  double deltat;               /* time_step[nts_prev].width */
  double tratmid;              /* time_step[nts].mid / tmin */
  double t_mid;                /* time_step[nts].mid: the bound-bound rates of the NLTE matrix (nltepop.cc:818) */
  double t_current_te;         /* time_step[nts - 1].mid: call_T_e_finder at titer 0 (update_grid.cc:804-806) */
  double tmin;
  double T_min, T_max;         /* MINTEMP, MAXTEMP */
  double accuracy;             /* TEMPERATURE_SOLVER_ACCURACY */
  double T_R_min, T_R_max;     /* bin fit range (artisoptions_nltenebular.h:109-110) */
} artis_nlte_params;

typedef struct artis_nlte_cells {
  int32_t ncells;
  int32_t pad0;
  const int32_t *mgi;                   /* [ncells] */
  /* inputs, indexed by mgi */
  const float *rho;                     /* grid::get_rho at this timestep */
  const float *elem_abundance, *elem_meanweight;  /* [npts_model * nelements] */
  const double *vol_init;
  const int16_t *thick;
  const double *deposition_rate_density;/* nonthermal::calculate_deposition_rate_density (nonthermal.cc:626-657) */
  /* raw estimators of the transport step (summed over ranks; the arrays of artis_estimators) */
  const double *J, *nuJ, *ffheating, *colheating;
  const double *bfrate_raw;             /* [npts_model * nbfcontinua] */
  const double *bin_J_raw, *bin_nuJ_raw;/* [npts_model * radfield_nbins] */
  const int64_t *bin_contribcount;
  /* in: the previous timestep's state; out: this timestep's (the artis_cell_state arrays the transport reads) */
  float *TR, *W, *TJ, *Te, *nne, *nnetot;
  float *groundlevelpop, *partfunct;    /* [npts_model * nions_total] */
  double *nlte_pops;                    /* [npts_model * total_nlte_levels] */
  float *bin_TR, *bin_W;                /* [npts_model * radfield_nbins] radfieldbin_solutions */
  float *bfrate_estimator;              /* [npts_model * nbfcontinua] prev_bfrate_normed */
  /* the non-thermal solution (nt_solution[mgi], nonthermal.cc:123-146), in / out */
  float *nt_frac_heating, *nt_frac_ionization, *nt_frac_excitation;   /* [npts_model] */
  float *nt_nneperion_when_solved;      /* [npts_model] */
  int32_t *nt_timestep_last_solved;     /* [npts_model] */
  float *nt_eff_ionpot;                 /* [npts_model * nions_total] */
  double *nt_fracdep_ionization_ion;    /* [npts_model * nions_total] */
  float *nt_prob_num_auger, *nt_ionenfrac_num_auger;  /* [npts_model * nions_total * (ARTIS_NT_MAX_AUGER + 1)] */
  /* outputs */
  double *nt_ionization_ratecoeff;      /* [npts_model * nions_total] nt_ionization_ratecoeff (nonthermal.cc:1684) */
  double *totalcooling, *cooling_contrib_ion;
  double *heatingcoolingrates;          /* [npts_model * ARTIS_TE_NRATES]; may be NULL */
  int32_t *nlte_iterations;             /* [npts_model] passes of the solve_Te_nltepops loop (0: LTE branch);
                                           may be NULL */
} artis_nlte_cells;
int artis_gpu_update_grid_nlte(const artis_nt_shells *nt, const artis_nlte_params *params, artis_nlte_cells *cells);
double artis_gpu_last_nlte_ms(void);  /* device time (ms) of the last artis_gpu_update_grid_nlte */

#define ARTIS_GPU_ABI_VERSION 11 /* 2: gamma / pellet / non-thermal path (artis_gamma_spectra and appended fields);
                                    3: virtual packets (artis_vpkt_params / artis_vpkt_result);
                                    4: artis_run_params.excitation_temperature;
                                    5: host estimator block pack/unpack, RCCL communicator + all-reduce;
                                    6: the nebular path (NLTE / superlevel populations, binned radiation field,
                                       detailed bf estimators, NO_LUT photoionisation, non-thermal ionisation);
                                    7: update_grid's temperature / ionisation solution (artis_gpu_solve_temperatures);
                                    8: update_grid for the nebular options (artis_gpu_update_grid_nlte),
                                       artis_te_params.direct_col_heat;
                                    9: artis_gpu_table_info (per-cell table budgets), artis_gpu_vpkt_last_drains
                                       (bounded virtual-packet spawn buffer);
                                   10: Compton / pair-production emissivity estimators (artis_run_params.comp_est,
                                       artis_estimators.compton_emiss, a section of the estimator block);
                                   11: artis_gpu_init refuses unsupported option values; rlc_emiss_rpkt into
                                       rpkt_emiss for do_rlc_est 1 / 2; artis_gpu_table_info's level-mode entries */
int artis_gpu_abi_version(void);

#ifdef __cplusplus
}
#endif

#endif /* ARTIS_GPU_H */
