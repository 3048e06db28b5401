"""ctypes mirrors of the C-ABI structs in include/artis_gpu.h and model_synth.h.

Plain data plumbing: every struct here has the same field order and types as the C header, and
tests/test_abi.py checks sizes/offsets against the compiled libraries.
"""
import ctypes as C
import os

import numpy as np

ARTIS_WORK_COUNT = 16
ARTIS_COUNTER_COUNT = 34
COMM_ID_BYTES = 128

TYPE_ESCAPE = 32
TYPE_RADIOACTIVE_PELLET = 100
TYPE_GAMMA = 10
TYPE_RPKT = 11
TYPE_KPKT = 12
TYPE_MA = 13
TYPE_NTLEPTON = 20
TYPE_NONTHERMAL_PREDEPOSIT = 21
TYPE_PRE_KPKT = 120

# reference struct packet (packet.h:28-73), 304 bytes; padding named (as in include/artis_gpu.h) so that
# the dtype has no gaps and numpy copies are byte-exact
PACKET_DTYPE = np.dtype(
    {
        "names": [
            "where", "type", "last_cross", "interactions", "nscatterings", "last_event",
            "pos", "dir", "e_cmf", "e_rf", "nu_cmf", "nu_rf", "next_trans", "emissiontype",
            "em_pos", "em_time", "_pad0", "prop_time", "absorptiontype", "trueemissiontype", "trueem_time", "_pad1",
            "absorptionfreq", "absorptiondir", "stokes", "pol_dir", "tdecay", "escape_type",
            "escape_time", "scat_count", "number", "originated_from_particlenotgamma", "_pad2",
            "pellet_decaytype", "pellet_nucindex", "trueemissionvelocity", "mastate",
        ],
        "formats": [
            "<i4", "<i4", "<i4", "<i4", "<i4", "<i4",
            ("<f8", 3), ("<f8", 3), "<f8", "<f8", "<f8", "<f8", "<i4", "<i4",
            ("<f8", 3), "<i4", "<i4", "<f8", "<i4", "<i4", "<i4", "<i4",
            "<f8", ("<f8", 3), ("<f8", 3), ("<f8", 3), "<f8", "<i4",
            "<i4", "<i4", "<i4", "u1", ("u1", 3),
            "<i4", "<i4", "<f4", ("<i4", 4),
        ],
        "offsets": [
            0, 4, 8, 12, 16, 20,
            24, 48, 72, 80, 88, 96, 104, 108,
            112, 136, 140, 144, 152, 156, 160, 164,
            168, 176, 200, 224, 248, 256,
            260, 264, 268, 272, 273,
            276, 280, 284, 288,
        ],
        "itemsize": 304,
    }
)

# work-counter indices (include/artis_constants.h enum artis_work)
WORK_NAMES = [
    "packets_active", "rpkt_steps", "lines_scanned", "line_taus", "kappa_evals", "bf_active",
    "est_segments", "gc_updates", "ma_jumps", "ma_trans", "kpkt", "kpkt_terms", "escaped",
    "es_scat", "bb_events", "cont_events",
]


class RunParams(C.Structure):
    _fields_ = [
        ("seed", C.c_uint32),
        ("rank", C.c_int32),
        ("opacity_case", C.c_int32),
        ("do_r_lc", C.c_int32),
        ("do_rlc_est", C.c_int32),
        ("n_kpktdiffusion_timesteps", C.c_int32),
        ("kpktdiffusion_timescale", C.c_float),
        ("max_path_step", C.c_double),
        ("pol_dipole", C.c_int32),
        ("relativistic_doppler", C.c_int32),
        ("record_linestat", C.c_int32),
        ("gamma_grey", C.c_double),
        ("instant_particle_deposition", C.c_int32),
        ("nt_solve_spencerfano", C.c_int32),
        ("excitation_temperature", C.c_int32),
        # ABI 6: the nebular options
        ("nlte_pops_on", C.c_int32),
        ("multibin_radfield", C.c_int32),
        ("first_nlte_radfield_timestep", C.c_int32),
        ("detailed_bf_estimators", C.c_int32),
        ("detailed_bf_usefromtimestep", C.c_int32),
        ("no_lut_photoion", C.c_int32),
        ("no_lut_bfheating", C.c_int32),
        ("nt_on", C.c_int32),
        ("nt_max_auger_electrons", C.c_int32),
        ("minpop", C.c_double),
        # ABI 10: Compton / pair-production emissivity estimators (emissivities.cc:14-136)
        ("comp_est", C.c_int32),
        ("emiss_offset", C.c_int32),
        ("emiss_max", C.c_int32),
        ("_pad_comp", C.c_int32),
        ("time_syn_first", C.c_double),
        ("time_syn_last", C.c_double),
        ("syn_dir", C.c_double * 3),
    ]


EMISS_MAX = 2  # ARTIS_EMISS_MAX (globals.h:223)
TEXC_TJ = 0
TEXC_TE = 1


class Estimators(C.Structure):
    _fields_ = [
        ("J", C.POINTER(C.c_double)),
        ("nuJ", C.POINTER(C.c_double)),
        ("ffheatingestimator", C.POINTER(C.c_double)),
        ("colheatingestimator", C.POINTER(C.c_double)),
        ("gammaestimator", C.POINTER(C.c_double)),
        ("bfheatingestimator", C.POINTER(C.c_double)),
        ("ecounter", C.POINTER(C.c_int32)),
        ("acounter", C.POINTER(C.c_int32)),
        ("cmf_lum", C.c_double),
        ("gamma_dep", C.c_double),
        ("positron_dep", C.c_double),
        ("electron_dep", C.c_double),
        ("electron_emission", C.c_double),
        ("alpha_dep", C.c_double),
        ("alpha_emission", C.c_double),
        ("gamma_emission", C.c_double),
        ("pellet_decays", C.c_int64),
        ("nesc", C.c_int64),
        ("counters", C.c_int64 * ARTIS_COUNTER_COUNT),
        ("rpkt_emiss", C.POINTER(C.c_double)),
        ("nt_energy_deposited", C.c_double),
        # ABI 6 (NULL unless the nebular options are on)
        ("bfrate_raw", C.POINTER(C.c_double)),
        ("radfield_J_raw", C.POINTER(C.c_double)),
        ("radfield_nuJ_raw", C.POINTER(C.c_double)),
        ("radfield_contribcount", C.POINTER(C.c_int64)),
        # ABI 10
        ("compton_emiss", C.POINTER(C.c_float)),
    ]


class SynthConfig(C.Structure):
    _fields_ = [
        ("ngrid_1d", C.c_int32),
        ("nshells_1d", C.c_int32),
        ("nlevels_per_ion", C.c_int32),
        ("n_ionising", C.c_int32),
        ("max_lines", C.c_int32),
        ("line_window", C.c_int32),
        ("n_resonance", C.c_int32),
        ("ntstep", C.c_int32),
        ("tmin_days", C.c_double),
        ("tmax_days", C.c_double),
        ("vmax", C.c_double),
        ("mass_msun", C.c_double),
        ("v_e", C.c_double),
        ("T0", C.c_double),
        ("n_tclasses", C.c_int32),
        ("seed", C.c_uint64),
        ("ionpot_scale", C.c_double),
        ("thick_tau", C.c_double),
        ("relativistic", C.c_int32),
        ("instant_particle_deposition", C.c_int32),
        ("n_kpktdiffusion_timesteps", C.c_int32),
        ("kpktdiffusion_timescale", C.c_double),
        ("excitation_te", C.c_int32),
        ("tj_scale", C.c_double),
        ("nebular", C.c_int32),
        ("nlte_level_max", C.c_int32),
        ("radfield_nbins", C.c_int32),
        ("first_nlte_radfield_timestep", C.c_int32),
        ("detailed_bf_usefromtimestep", C.c_int32),
        ("minpop", C.c_double),
        ("nu_min_r", C.c_double),
        ("nu_max_r", C.c_double),
        ("grid_spherical", C.c_int32),
    ]


class GammaSpectra(C.Structure):
    _fields_ = [
        ("nnuclides", C.c_int32),
        ("nuc_nlines", C.POINTER(C.c_int32)),
        ("nuc_line_offset", C.POINTER(C.c_int32)),
        ("nuc_endecay_gamma", C.POINTER(C.c_double)),
        ("line_energy", C.POINTER(C.c_double)),
        ("line_probability", C.POINTER(C.c_double)),
    ]


class EstimatorArrays:
    """Host-side numpy storage for one artis_estimators block (reference zero_estimators shapes)."""

    def __init__(self, npts_model, nelements, maxnions, nlines, nbfcontinua=0, radfield_nbins=0):
        """nbfcontinua > 0: bfrate_raw (DETAILED_BF_ESTIMATORS_ON); radfield_nbins > 0: the bin estimators
        (MULTIBIN_RADFIELD_MODEL_ON)."""
        self.npts_model, self.nelements, self.maxnions = npts_model, nelements, maxnions
        self.nbfcontinua, self.radfield_nbins = nbfcontinua, radfield_nbins
        self.J = np.zeros(npts_model)
        self.nuJ = np.zeros(npts_model)
        self.ffheating = np.zeros(npts_model)
        self.colheating = np.zeros(npts_model)
        self.gamma = np.zeros(npts_model * nelements * maxnions)
        self.bfheating = np.zeros(npts_model * nelements * maxnions)
        self.ecounter = np.zeros(nlines, dtype=np.int32)
        self.acounter = np.zeros(nlines, dtype=np.int32)
        self.rpkt_emiss = np.zeros(npts_model)
        self.struct = Estimators()
        dp = lambda a: a.ctypes.data_as(C.POINTER(C.c_double))  # noqa: E731
        ip = lambda a: a.ctypes.data_as(C.POINTER(C.c_int32))  # noqa: E731
        s = self.struct
        s.J, s.nuJ = dp(self.J), dp(self.nuJ)
        s.ffheatingestimator, s.colheatingestimator = dp(self.ffheating), dp(self.colheating)
        s.gammaestimator, s.bfheatingestimator = dp(self.gamma), dp(self.bfheating)
        s.ecounter, s.acounter = ip(self.ecounter), ip(self.acounter)
        s.rpkt_emiss = dp(self.rpkt_emiss)
        # globals::compton_emiss [(npts_model + 1) * EMISS_MAX] floats (grid.cc:1699)
        self.compton_emiss = np.zeros((npts_model + 1) * EMISS_MAX, dtype=np.float32)
        s.compton_emiss = self.compton_emiss.ctypes.data_as(C.POINTER(C.c_float))
        self.bfrate_raw = np.zeros(npts_model * nbfcontinua)
        self.radfield_J = np.zeros(npts_model * radfield_nbins)
        self.radfield_nuJ = np.zeros(npts_model * radfield_nbins)
        self.radfield_count = np.zeros(npts_model * radfield_nbins, dtype=np.int64)
        if nbfcontinua > 0:
            s.bfrate_raw = dp(self.bfrate_raw)
        if radfield_nbins > 0:
            s.radfield_J_raw, s.radfield_nuJ_raw = dp(self.radfield_J), dp(self.radfield_nuJ)
            s.radfield_contribcount = self.radfield_count.ctypes.data_as(C.POINTER(C.c_int64))

    @property
    def counters(self):
        return np.array(self.struct.counters[:], dtype=np.int64)

    def scalars(self):
        s = self.struct
        return {
            "cmf_lum": s.cmf_lum,
            "gamma_dep": s.gamma_dep,
            "positron_dep": s.positron_dep,
            "electron_dep": s.electron_dep,
            "electron_emission": s.electron_emission,
            "alpha_dep": s.alpha_dep,
            "alpha_emission": s.alpha_emission,
            "gamma_emission": s.gamma_emission,
            "pellet_decays": s.pellet_decays,
            "nt_energy_deposited": s.nt_energy_deposited,
            "nesc": s.nesc,
        }


# virtual packets (include/artis_gpu.h artis_vpkt_params / artis_vpkt_result; vpkt.cc, vpkt.h:30-47)
VPKT_MAX_SPECTRA = 8
VPKT_MRANGE = 4
VPKT_MRANGE_GRID = 5
DAY = 86400.0
CLIGHT = 2.99792458e10


class VpktParams(C.Structure):
    _fields_ = [
        ("nobs", C.c_int32),
        ("nz_obs", C.POINTER(C.c_double)),
        ("phi_obs", C.POINTER(C.c_double)),
        ("nspectra", C.c_int32),
        ("exclude", C.POINTER(C.c_double)),
        ("tmin_vspec", C.c_double),
        ("tmax_vspec", C.c_double),
        ("numin_vspec", C.c_double),
        ("numax_vspec", C.c_double),
        ("vmtbins", C.c_int32),
        ("vmnubins", C.c_int32),
        ("tmin_vspec_input", C.c_double),
        ("tmax_vspec_input", C.c_double),
        ("nrange", C.c_int32),
        ("numin_vspec_input", C.c_double * VPKT_MRANGE),
        ("numax_vspec_input", C.c_double * VPKT_MRANGE),
        ("tau_max_vpkt", C.c_double),
        ("vgrid_flag", C.c_int32),
        ("tmin_grid", C.c_double),
        ("tmax_grid", C.c_double),
        ("nrange_grid", C.c_int32),
        ("nu_grid_min", C.c_double * VPKT_MRANGE_GRID),
        ("nu_grid_max", C.c_double * VPKT_MRANGE_GRID),
        ("ny_vgrid", C.c_int32),
        ("nz_vgrid", C.c_int32),
        ("nprocs", C.c_int32),
        ("spawn_capacity", C.c_int64),
    ]


class VpktResult(C.Structure):
    _fields_ = [
        ("vstokes_i", C.POINTER(C.c_double)),
        ("vstokes_q", C.POINTER(C.c_double)),
        ("vstokes_u", C.POINTER(C.c_double)),
        ("vgrid_i", C.POINTER(C.c_double)),
        ("vgrid_q", C.POINTER(C.c_double)),
        ("vgrid_u", C.POINTER(C.c_double)),
        ("nvpkt", C.c_int64),
        ("nvpkt_esc1", C.c_int64),
        ("nvpkt_esc2", C.c_int64),
        ("nvpkt_esc3", C.c_int64),
    ]


class VpktConfig:
    """vpkt.txt parameters (read_parameterfile_vpkt, vpkt.cc:667-835) with the vpkt.h compile-time binning as
    defaults; `struct` is the artis_vpkt_params view (the numpy arrays it points to are kept alive here)."""

    def __init__(self, nz_obs=(0.5,), phi_obs_deg=(0.0,), exclude=(0.0,), tmin_days=10.0, tmax_days=30.0,
                 lambda_min=3500.0, lambda_max=10000.0, vmtbins=30, vmnubins=2500, tmin_input_days=None,
                 tmax_input_days=None, ranges_angstrom=None, tau_max=10.0, vgrid=False, grid_tmin_days=None,
                 grid_tmax_days=None, grid_ranges_angstrom=((3500.0, 10000.0),), ny_vgrid=50, nz_vgrid=50, nprocs=1,
                 spawn_capacity=0):
        nz = np.array(nz_obs, dtype=np.float64)
        nz[nz == 1] = 0.9999  # vpkt.cc:683-687
        nz[nz == -1] = -0.9999
        self.nz_obs = np.ascontiguousarray(nz)
        self.phi_obs = np.ascontiguousarray(np.array(phi_obs_deg, dtype=np.float64) * np.pi / 180.0)
        self.exclude = np.ascontiguousarray(np.array(exclude, dtype=np.float64))
        assert len(self.nz_obs) == len(self.phi_obs) and len(self.exclude) <= VPKT_MAX_SPECTRA
        s = VpktParams()
        dp = lambda a: a.ctypes.data_as(C.POINTER(C.c_double))  # noqa: E731
        s.nobs = len(self.nz_obs)
        s.nz_obs, s.phi_obs = dp(self.nz_obs), dp(self.phi_obs)
        s.nspectra = len(self.exclude)
        s.exclude = dp(self.exclude)
        s.tmin_vspec, s.tmax_vspec = tmin_days * DAY, tmax_days * DAY
        s.numin_vspec = CLIGHT / lambda_max * 1e8  # vpkt.h:36-37
        s.numax_vspec = CLIGHT / lambda_min * 1e8
        s.vmtbins, s.vmnubins = vmtbins, vmnubins
        s.tmin_vspec_input = (tmin_input_days if tmin_input_days is not None else tmin_days) * DAY
        s.tmax_vspec_input = (tmax_input_days if tmax_input_days is not None else tmax_days) * DAY
        if ranges_angstrom is None:
            s.nrange = 1
            s.numin_vspec_input[0], s.numax_vspec_input[0] = s.numin_vspec, s.numax_vspec
        else:
            s.nrange = len(ranges_angstrom)
            for i, (lmin, lmax) in enumerate(ranges_angstrom):  # vpkt.cc:767-768
                s.numin_vspec_input[i] = CLIGHT / (lmax * 1e-8)
                s.numax_vspec_input[i] = CLIGHT / (lmin * 1e-8)
        s.tau_max_vpkt = tau_max
        s.vgrid_flag = 1 if vgrid else 0
        s.tmin_grid = (grid_tmin_days if grid_tmin_days is not None else tmin_days) * DAY
        s.tmax_grid = (grid_tmax_days if grid_tmax_days is not None else tmax_days) * DAY
        s.nrange_grid = len(grid_ranges_angstrom) if vgrid else 0
        for i, (lmin, lmax) in enumerate(grid_ranges_angstrom if vgrid else ()):  # vpkt.cc:826-827
            s.nu_grid_max[i] = CLIGHT / (lmin * 1e-8)
            s.nu_grid_min[i] = CLIGHT / (lmax * 1e-8)
        s.ny_vgrid, s.nz_vgrid = ny_vgrid, nz_vgrid
        s.nprocs = nprocs
        s.spawn_capacity = spawn_capacity
        self.struct = s

    @property
    def nobs(self):
        return self.struct.nobs

    @property
    def nspectra(self):
        return self.struct.nspectra

    def bins(self):
        """init_vspecpol (vpkt.cc:425-436): float32 lower_time/delta_t [vmtbins], lower_freq/delta_freq [vmnubins]."""
        s = self.struct
        dlogt = (np.log(s.tmax_vspec) - np.log(s.tmin_vspec)) / s.vmtbins
        dlognu = (np.log(s.numax_vspec) - np.log(s.numin_vspec)) / s.vmnubins
        n = np.arange(s.vmtbins)
        lt = np.exp(np.log(s.tmin_vspec) + n * dlogt).astype(np.float32)
        dt = (np.exp(np.log(s.tmin_vspec) + (n + 1) * dlogt) - lt.astype(np.float64)).astype(np.float32)
        m = np.arange(s.vmnubins)
        lf = np.exp(np.log(s.numin_vspec) + m * dlognu).astype(np.float32)
        df = (np.exp(np.log(s.numin_vspec) + (m + 1) * dlognu) - lf.astype(np.float64)).astype(np.float32)
        return lt, dt, lf, df


class VpktArrays:
    """Host storage for one artis_vpkt_result: vstokes [3][vmtbins][nobs*nspectra][vmnubins], vgrid
    [3][ny][nz][nrange_grid][nobs]."""

    def __init__(self, cfg):
        s = cfg.struct
        self.vstokes = np.zeros((3, s.vmtbins, s.nobs * s.nspectra, s.vmnubins))
        ng = max(s.nrange_grid, 1)
        self.vgrid = np.zeros((3, s.ny_vgrid, s.nz_vgrid, ng, s.nobs))
        self.struct = VpktResult()
        dp = lambda a: a.ctypes.data_as(C.POINTER(C.c_double))  # noqa: E731
        r = self.struct
        r.vstokes_i, r.vstokes_q, r.vstokes_u = dp(self.vstokes[0]), dp(self.vstokes[1]), dp(self.vstokes[2])
        r.vgrid_i, r.vgrid_q, r.vgrid_u = dp(self.vgrid[0]), dp(self.vgrid[1]), dp(self.vgrid[2])

    def counters(self):
        r = self.struct
        return {"nvpkt": r.nvpkt, "nvpkt_esc1": r.nvpkt_esc1, "nvpkt_esc2": r.nvpkt_esc2, "nvpkt_esc3": r.nvpkt_esc3}


# exspec spectra (include/artis_gpu.h artis_spectra_request / artis_spectra_out)
MABINS = 100


class SpectraRequest(C.Structure):
    _fields_ = [("nnubins", C.c_int32), ("nprocs", C.c_int32), ("abin", C.c_int32), ("syn_dir", C.c_double * 3)]


class SpectraOut(C.Structure):
    _fields_ = [(n, C.POINTER(C.c_double)) for n in (
        "flux", "emission", "trueemission", "absorption", "stokes_flux", "stokes_emission", "stokes_absorption",
        "lc_lum", "lc_lumcmf", "gamma_lc_lum", "gamma_lc_lumcmf")]


class SpectraArrays:
    """Host storage of one artis_spectra_out: flux [ntstep, nnubins]; emission / trueemission
    [ntstep, nnubins, proccount]; absorption [ntstep, nnubins, ioncount]; stokes_* with a leading axis of 3
    (I, Q, U); light curves [ntstep]."""

    def __init__(self, ntstep, nnubins, nelements, maxnions, emission_res=True, stokes=False):
        self.ioncount = nelements * maxnions
        self.proccount = 2 * self.ioncount + 1
        self.nnubins = nnubins
        z = np.zeros
        self.flux = z((ntstep, nnubins))
        self.emission = z((ntstep, nnubins, self.proccount)) if emission_res else None
        self.trueemission = z((ntstep, nnubins, self.proccount)) if emission_res else None
        self.absorption = z((ntstep, nnubins, self.ioncount)) if emission_res else None
        self.stokes_flux = z((3, ntstep, nnubins)) if stokes else None
        self.stokes_emission = z((3, ntstep, nnubins, self.proccount)) if stokes and emission_res else None
        self.stokes_absorption = z((3, ntstep, nnubins, self.ioncount)) if stokes and emission_res else None
        self.lc_lum, self.lc_lumcmf = z(ntstep), z(ntstep)
        self.gamma_lc_lum, self.gamma_lc_lumcmf = z(ntstep), z(ntstep)
        self.struct = SpectraOut()
        for name, _ in SpectraOut._fields_:
            a = getattr(self, name)
            if a is not None:
                setattr(self.struct, name, a.ctypes.data_as(C.POINTER(C.c_double)))

    def arrays(self):
        return {n: getattr(self, n) for n, _ in SpectraOut._fields_ if getattr(self, n) is not None}


def spectra_request(nnubins=1000, nprocs=1, abin=-1, syn_dir=(0., 0., 1.)):
    r = SpectraRequest()
    r.nnubins, r.nprocs, r.abin = nnubins, nprocs, abin
    for k in range(3):
        r.syn_dir[k] = syn_dir[k]
    return r


# update_grid's temperature / ionisation solution (include/artis_gpu.h artis_te_*; ABI 7)
TE_NRATES = 8
TE_RATE_NAMES = ["cooling_collisional", "cooling_fb", "cooling_ff", "cooling_adiabatic", "heating_collisional",
                 "heating_bf", "heating_ff", "heating_dep"]


class TeTables(C.Structure):
    _fields_ = [("bfheating_coeff", C.c_void_p), ("ion_alpha_sp", C.c_void_p)]


class TeParams(C.Structure):
    _fields_ = [("t_current", C.c_double), ("tmin", C.c_double), ("T_min", C.c_double), ("T_max", C.c_double),
                ("accuracy", C.c_double), ("initial_iteration", C.c_int32), ("direct_col_heat", C.c_int32)]


_TE_CELL_PTRS = ["mgi", "TR", "W", "TJ", "rho", "thick", "elem_abundance", "elem_meanweight", "vol_init",
                 "ffheatingestimator", "colheatingestimator", "gammaestimator", "bfheatingestimator", "heating_dep",
                 "Te", "groundlevelpop", "nne", "nnetot", "partfunct", "totalcooling", "cooling_contrib_ion",
                 "heatingcoolingrates", "te_iterations"]


class TeCells(C.Structure):
    _fields_ = [("ncells", C.c_int32), ("pad0", C.c_int32)] + [(n, C.c_void_p) for n in _TE_CELL_PTRS]


class CellState(C.Structure):
    """artis_cell_state (read-only view of a model's update_grid outputs)."""
    _fields_ = [(n, C.c_void_p) for n in ("Te", "TR", "TJ", "W", "nne", "nnetot", "rho", "kappagrey", "thick",
                                           "elem_abundance", "groundlevelpop", "partfunct", "totalcooling",
                                           "cooling_contrib_ion", "corrphotoionrenorm", "ffegrp", "nlte_pops",
                                           "radfield_bin_TR", "radfield_bin_W", "bfrate_estimator",
                                           "nt_deposition_rate_density", "nt_ionization_ratecoeff",
                                           "nt_prob_num_auger", "nt_ionenfrac_num_auger")]


class AtomicHeader(C.Structure):
    """The leading fields of artis_atomic_tables (counts, LUT grid, element arrays)."""
    _fields_ = [("nelements", C.c_int32), ("maxnions", C.c_int32), ("nions_total", C.c_int32),
                ("nlevels_total", C.c_int32), ("nlines", C.c_int32), ("nbfcontinua", C.c_int32),
                ("nbfcontinua_ground", C.c_int32), ("ncoolingterms", C.c_int32), ("nphixspoints", C.c_int32),
                ("nphixsnuincrement", C.c_double), ("last_phixs_nuovernuedge", C.c_double),
                ("phixs_file_version", C.c_int32), ("tablesize", C.c_int32), ("mintemp", C.c_double),
                ("maxtemp", C.c_double), ("elem_anumber", C.c_void_p), ("elem_nions", C.c_void_p),
                ("elem_uniqueionoffset", C.c_void_p)]


MH = 1.67352e-24


class TeArrays:
    """Host storage for one artis_te_cells block: the update_grid inputs of a model's non-empty cells (its current
    cell state as the previous timestep's solution) plus synthetic normalised heating / photoionisation estimators
    (seeded), and the output arrays.  The same block feeds the engine and the oracle."""

    def __init__(self, model, t_current, seed=3, thick_frac=0.0, lte_all=False, gamma_zero_frac=0.1, synthetic=True):
        """synthetic=False: the estimator inputs are left zero for the caller to fill (the timestep loop's own
        prepared estimators), without drawing the seeded stand-ins."""
        m = model
        cs = CellState.from_address(m.cellstate)
        hdr = AtomicHeader.from_address(m.atomic)
        np_, nel, ni, mx = m.npts_model, m.nelements, m.nions_total, m.maxnions
        f32 = lambda p, n: np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_float)), (n,)).copy()  # noqa: E731
        self.TR, self.W, self.TJ = f32(cs.TR, np_), f32(cs.W, np_), f32(cs.TJ, np_)
        self.rho = f32(cs.rho, np_)
        self.Te = f32(cs.Te, np_)
        self.elem_abundance = f32(cs.elem_abundance, np_ * nel)
        self.groundlevelpop = f32(cs.groundlevelpop, np_ * ni)
        anum = np.ctypeslib.as_array(C.cast(hdr.elem_anumber, C.POINTER(C.c_int32)), (nel,)).copy()
        # initstablemeannucmass stand-in: A ~ 2.1 Z nucleons
        self.elem_meanweight = np.tile((2.1 * anum * MH).astype(np.float32), np_)
        self.vol_init = np.full(np_, 1e45)
        self.mgi_list = np.nonzero(self.rho > 0)[0].astype(np.int32)
        if synthetic:
            rng = np.random.default_rng(seed)
            self.thick = (rng.random(np_) < thick_frac).astype(np.int16)
            if lte_all:
                self.thick[:] = 1
            # normalised estimators: heating terms of the order of the cell's LTE bf heating, spread per cell
            self.ffheating = 10 ** rng.uniform(-12, -9, np_) * self.rho / 1e-14
            self.colheating = 10 ** rng.uniform(-12, -9, np_) * self.rho / 1e-14
            cell_scale = np.repeat(10 ** rng.uniform(-1.5, 3.0, np_), nel * mx)  # some cells balance inside [T_min, T_max]
            self.bfheating = cell_scale * 10 ** rng.uniform(-0.3, 0.3, np_ * nel * mx)
            self.gamma = 10 ** rng.uniform(-4., 1., np_ * nel * mx)
            self.gamma[rng.random(np_ * nel * mx) < gamma_zero_frac] = 0.
        else:
            self.thick = np.zeros(np_, np.int16)
            self.ffheating, self.colheating = np.zeros(np_), np.zeros(np_)
            self.bfheating, self.gamma = np.zeros(np_ * nel * mx), np.zeros(np_ * nel * mx)
        self.heating_dep = None
        self.nne = np.zeros(np_, np.float32)
        self.nnetot = np.zeros(np_, np.float32)
        self.partfunct = np.zeros(np_ * ni, np.float32)
        self.totalcooling = np.zeros(np_)
        self.cooling_contrib_ion = np.zeros(np_ * ni)
        self.rates = np.zeros(np_ * TE_NRATES)
        self.iters = np.zeros(np_, np.int32)
        self.params = TeParams(t_current=float(t_current), tmin=float(m.cfg.tmin_days) * 86400.0,
                               T_min=float(hdr.mintemp), T_max=float(hdr.maxtemp), accuracy=1e-2,
                               initial_iteration=0)
        self.tables = C.c_void_p(model._lib.artis_model_te_tables(model._h))

    def struct(self):
        s = TeCells()
        s.ncells = len(self.mgi_list)
        for n, a in (("mgi", self.mgi_list), ("TR", self.TR), ("W", self.W), ("TJ", self.TJ), ("rho", self.rho),
                     ("thick", self.thick), ("elem_abundance", self.elem_abundance),
                     ("elem_meanweight", self.elem_meanweight), ("vol_init", self.vol_init),
                     ("ffheatingestimator", self.ffheating), ("colheatingestimator", self.colheating),
                     ("gammaestimator", self.gamma), ("bfheatingestimator", self.bfheating), ("Te", self.Te),
                     ("groundlevelpop", self.groundlevelpop), ("nne", self.nne), ("nnetot", self.nnetot),
                     ("partfunct", self.partfunct), ("totalcooling", self.totalcooling),
                     ("cooling_contrib_ion", self.cooling_contrib_ion), ("heatingcoolingrates", self.rates),
                     ("te_iterations", self.iters)):
            setattr(s, n, a.ctypes.data)
        if self.heating_dep is not None:
            s.heating_dep = self.heating_dep.ctypes.data
        return s

    def copy(self):
        import copy as _c
        o = _c.copy(self)
        for k, v in self.__dict__.items():
            if isinstance(v, np.ndarray):
                setattr(o, k, v.copy())
        return o


class UgPrepare(C.Structure):
    """artis_ug_prepare (ABI 7): update_grid_cell's estimator preparation."""
    _fields_ = [("deltat", C.c_double), ("tratmid", C.c_double), ("nprocs", C.c_int32), ("pad0", C.c_int32)] + [
        (n, C.c_void_p) for n in ("J", "nuJ", "ffheating", "colheating", "gammaestimator", "bfheatingestimator", "nne",
                                  "partfunct", "TR_out", "W_out", "TJ_out", "ffheating_out", "colheating_out",
                                  "gamma_out", "bfheating_out", "corrphotoionrenorm_out")]


class UgArrays:
    """Raw transport estimators for artis_ug_prepare (seeded, of the magnitude a 1e4-packet step accumulates per cell
    of a small model) plus the previous n_e / partition functions of the model's cell state, and the outputs."""

    def __init__(self, model, deltat, tratmid, seed=6, synthetic=True):
        """synthetic=False: the raw estimators are left zero for the caller to fill (the timestep loop's own)."""
        m = model
        cs = CellState.from_address(m.cellstate)
        np_, nel, ni, mx = m.npts_model, m.nelements, m.nions_total, m.maxnions
        f32 = lambda p, n: np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_float)), (n,)).copy()  # noqa: E731
        self.deltat, self.tratmid, self.nprocs = float(deltat), float(tratmid), 1
        self.nne = f32(cs.nne, np_)
        self.partfunct = f32(cs.partfunct, np_ * ni)
        if synthetic:
            rng = np.random.default_rng(seed)
            # J ~ 4 pi sigma T^4 / pi * volume * deltat, with nubar giving T_R ~ 5000-15000 K
            T = rng.uniform(5e3, 1.5e4, np_)
            self.J = 4 * np.pi * 5.6704e-5 * T ** 4 / np.pi * 1e45 * deltat * rng.uniform(0.5, 1.5, np_)
            self.nuJ = self.J * (1.38064852e-16 * 3.832229494 * T * rng.uniform(0.8, 1.2, np_) / 6.6260755e-27)
            self.ffheating = self.J * 1e-18
            self.colheating = self.J * 1e-17
            self.gamma = self.J.repeat(nel * mx) * 10 ** rng.uniform(-22, -20, np_ * nel * mx)
            self.bfheating = self.J.repeat(nel * mx) * 10 ** rng.uniform(-20, -18, np_ * nel * mx)
        else:
            self.J, self.nuJ, self.ffheating, self.colheating = (np.zeros(np_) for _ in range(4))
            self.gamma, self.bfheating = np.zeros(np_ * nel * mx), np.zeros(np_ * nel * mx)
        self.TR_out = np.zeros(np_, np.float32)
        self.W_out = np.zeros(np_, np.float32)
        self.TJ_out = np.zeros(np_, np.float32)
        self.ff_out = np.zeros(np_)
        self.col_out = np.zeros(np_)
        self.gamma_out = np.zeros(np_ * nel * mx)
        self.bfheating_out = np.zeros(np_ * nel * mx)
        self.renorm_out = np.zeros(np_ * nel * mx)

    def struct(self):
        s = UgPrepare(deltat=self.deltat, tratmid=self.tratmid, nprocs=self.nprocs)
        for n, a in (("J", self.J), ("nuJ", self.nuJ), ("ffheating", self.ffheating), ("colheating", self.colheating),
                     ("gammaestimator", self.gamma), ("bfheatingestimator", self.bfheating), ("nne", self.nne),
                     ("partfunct", self.partfunct), ("TR_out", self.TR_out), ("W_out", self.W_out),
                     ("TJ_out", self.TJ_out), ("ffheating_out", self.ff_out), ("colheating_out", self.col_out),
                     ("gamma_out", self.gamma_out), ("bfheating_out", self.bfheating_out),
                     ("corrphotoionrenorm_out", self.renorm_out)):
            setattr(s, n, a.ctypes.data)
        return s


# ----------------------------------------------------------------------- update_grid for the nebular options (ABI 8)
NT_MAX_AUGER = 2  # ARTIS_NT_MAX_AUGER


class NtShells(C.Structure):
    """artis_nt_shells: the Spencer-Fano inputs of nonthermal::init (nonthermal.cc:183-437)."""
    _fields_ = [("nshells", C.c_int32), ("sfpts", C.c_int32), ("sf_emin", C.c_double), ("sf_emax", C.c_double)] + [
        (n, C.c_void_p) for n in ("Z", "nelec", "n", "l", "ionpot_ev", "A", "B", "C", "D", "prob_num_auger",
                                  "en_auger_ev", "electron_binding")]


class NtData(C.Structure):
    _fields_ = [("shells", NtShells), ("storage", C.c_void_p)]


class Geometry(C.Structure):
    """artis_geometry (include/artis_gpu.h)."""
    _fields_ = [("grid_type", C.c_int32), ("ncoordgrid", C.c_int32 * 3), ("ngrid", C.c_int32),
                ("npts_model", C.c_int32), ("cell_pos_min", C.POINTER(C.c_double)), ("cell_mgi", C.POINTER(C.c_int32)),
                ("modelcell_wid_init", C.POINTER(C.c_double)), ("coordmax", C.c_double * 3), ("tmin", C.c_double),
                ("tmax", C.c_double), ("rmax", C.c_double), ("vmax", C.c_double), ("ntstep", C.c_int32),
                ("ts_start", C.POINTER(C.c_double)), ("ts_width", C.POINTER(C.c_double)),
                ("ts_mid", C.POINTER(C.c_double)), ("nu_min_r", C.c_double), ("nu_max_r", C.c_double)]


class NlteParams(C.Structure):
    _fields_ = [("nts", C.c_int32), ("num_lte_timesteps", C.c_int32), ("initial_iteration", C.c_int32),
                ("nprocs", C.c_int32), ("nlteiter", C.c_int32), ("do_rlc_est", C.c_int32), ("deltat", C.c_double),
                ("tratmid", C.c_double), ("t_mid", C.c_double), ("t_current_te", C.c_double), ("tmin", C.c_double),
                ("T_min", C.c_double), ("T_max", C.c_double), ("accuracy", C.c_double), ("T_R_min", C.c_double),
                ("T_R_max", C.c_double)]


_NLTE_CELL_PTRS = ["mgi", "rho", "elem_abundance", "elem_meanweight", "vol_init", "thick", "deposition_rate_density",
                   "J", "nuJ", "ffheating", "colheating", "bfrate_raw", "bin_J_raw", "bin_nuJ_raw",
                   "bin_contribcount", "TR", "W", "TJ", "Te", "nne", "nnetot", "groundlevelpop", "partfunct",
                   "nlte_pops", "bin_TR", "bin_W", "bfrate_estimator", "nt_frac_heating", "nt_frac_ionization",
                   "nt_frac_excitation", "nt_nneperion_when_solved", "nt_timestep_last_solved", "nt_eff_ionpot",
                   "nt_fracdep_ionization_ion", "nt_prob_num_auger", "nt_ionenfrac_num_auger",
                   "nt_ionization_ratecoeff", "totalcooling", "cooling_contrib_ion", "heatingcoolingrates",
                   "nlte_iterations"]


class NlteCells(C.Structure):
    _fields_ = [("ncells", C.c_int32), ("pad0", C.c_int32)] + [(n, C.c_void_p) for n in _NLTE_CELL_PTRS]


def nt_data_dir():
    """The reference's data/ tables read by the Spencer-Fano setup (collion.txt, binding_energies.txt,
    auger-km1993-table2.txt), shipped as package data."""
    return os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "nt_data")


class NtDataHandle:
    """The Spencer-Fano inputs read by the host library (artis_read_nt_data) for a model's included ions."""

    def __init__(self, model, sfpts=4096, sf_emin=0.1, sf_emax=16000., datadir=None):
        from . import io as _io

        lib = _io.lib()
        lib.artis_read_nt_data.argtypes = [C.c_char_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int,
                                           C.c_double, C.c_double, C.POINTER(NtData)]
        lib.artis_free_nt_data.argtypes = [C.POINTER(NtData)]
        lib.artis_free_nt_data.restype = None
        self._lib = lib
        hdr = AtomicHeader.from_address(model.atomic)
        nel = model.nelements
        anum = np.ctypeslib.as_array(C.cast(hdr.elem_anumber, C.POINTER(C.c_int32)), (nel,)).copy()
        nions = np.ctypeslib.as_array(C.cast(hdr.elem_nions, C.POINTER(C.c_int32)), (nel,)).copy()
        uoff = np.ctypeslib.as_array(C.cast(hdr.elem_uniqueionoffset, C.POINTER(C.c_int32)), (nel,)).copy()
        ionstage_all = model.ion_ionstage()
        ionstage0 = np.array([ionstage_all[u] for u in uoff], dtype=np.int32)
        self.data = NtData()
        rc = lib.artis_read_nt_data((datadir or nt_data_dir()).encode(), nel, anum.ctypes.data, ionstage0.ctypes.data,
                                    nions.ctypes.data, int(sfpts), float(sf_emin), float(sf_emax),
                                    C.byref(self.data))
        if rc != 0:
            raise RuntimeError(f"artis_read_nt_data -> {rc}")
        self.shells = self.data.shells

    def __del__(self):
        try:
            self._lib.artis_free_nt_data(C.byref(self.data))
        except Exception:
            pass


GRID_UNIFORM, GRID_SPHERICAL1D = 1, 2


def model_vol_init(model):
    """vol_init_modelcell (grid.cc:94-110): the uniform grid's cell volume at tmin times the number of propagation
    cells mapped to each model cell; on the spherical grid the shell volume 4/3 pi (r_out^3 - r_in^3) at tmin."""
    g = Geometry.from_address(model.geometry)
    mgi = np.ctypeslib.as_array(g.cell_mgi, (g.ngrid,))
    if g.grid_type == GRID_SPHERICAL1D:
        r_in = np.ctypeslib.as_array(g.cell_pos_min, (g.ngrid * 3,))[0::3].copy()
        r_out = r_in + np.ctypeslib.as_array(g.modelcell_wid_init, (g.ngrid,))
        vol = 4. / 3. * np.pi * (r_out ** 3 - r_in ** 3)
        return np.where(mgi < g.npts_model, vol, 0.)[:g.npts_model]
    counts = np.bincount(mgi[mgi < g.npts_model], minlength=g.npts_model)[:g.npts_model]
    wid = [2 * g.coordmax[d] / g.ncoordgrid[d] for d in range(3)]
    return counts * (wid[0] * wid[1] * wid[2])


def model_time_grid(model):
    g = Geometry.from_address(model.geometry)
    n = g.ntstep
    return (np.ctypeslib.as_array(g.ts_start, (n,)).copy(), np.ctypeslib.as_array(g.ts_width, (n,)).copy(),
            np.ctypeslib.as_array(g.ts_mid, (n,)).copy(), g.tmin)


class NlteArrays:
    """Host storage for one artis_nlte_cells block: a nebular model's non-empty cells with its current cell state as
    the previous timestep's solution, the raw estimators of a transport step (an EstimatorArrays) or seeded ones, the
    non-thermal solution state and the outputs.  The same block feeds the engine and the oracle."""

    def __init__(self, model, nts, est=None, seed=3, thick_frac=0.0, initial_iteration=0, nprocs=1, dep_scale=1.0):
        m = model
        cs = CellState.from_address(m.cellstate)
        hdr = AtomicHeader.from_address(m.atomic)
        np_, nel, ni = m.npts_model, m.nelements, m.nions_total
        nb, nbf, ntl = m.radfield_nbins, m.nbfcontinua, m.total_nlte_levels
        f32 = lambda p, n: np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_float)), (n,)).copy()  # noqa: E731
        f64 = lambda p, n: np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_double)), (n,)).copy()  # noqa: E731
        rng = np.random.default_rng(seed)
        self.rho = f32(cs.rho, np_)
        self.elem_abundance = f32(cs.elem_abundance, np_ * nel)
        anum = np.ctypeslib.as_array(C.cast(hdr.elem_anumber, C.POINTER(C.c_int32)), (nel,)).copy()
        self.elem_meanweight = np.tile((2.1 * anum * MH).astype(np.float32), np_)
        self.vol_init = model_vol_init(m).astype(np.float64)
        self.thick = (rng.random(np_) < thick_frac).astype(np.int16)
        self.mgi_list = np.nonzero(self.rho > 0)[0].astype(np.int32)
        self.deposition_rate_density = f64(cs.nt_deposition_rate_density, np_) * dep_scale
        # the previous timestep's state
        self.TR, self.W, self.TJ, self.Te = (f32(getattr(cs, n), np_) for n in ("TR", "W", "TJ", "Te"))
        self.nne, self.nnetot = f32(cs.nne, np_), f32(cs.nnetot, np_)
        self.groundlevelpop, self.partfunct = f32(cs.groundlevelpop, np_ * ni), f32(cs.partfunct, np_ * ni)
        self.nlte_pops = f64(cs.nlte_pops, np_ * max(ntl, 1))
        self.bin_TR, self.bin_W = f32(cs.radfield_bin_TR, np_ * nb), f32(cs.radfield_bin_W, np_ * nb)
        self.bfrate_estimator = f32(cs.bfrate_estimator, np_ * max(nbf, 1))
        # nt_solution as nonthermal::init leaves it (nonthermal.cc:508-548)
        A1 = NT_MAX_AUGER + 1
        self.nt_frac_heating = np.full(np_, 0.97, np.float32)
        self.nt_frac_ionization = np.full(np_, 0.03, np.float32)
        self.nt_frac_excitation = np.zeros(np_, np.float32)
        self.nt_nneperion_when_solved = np.full(np_, -1., np.float32)
        self.nt_timestep_last_solved = np.full(np_, -1, np.int32)
        self.nt_eff_ionpot = np.zeros(np_ * ni, np.float32)
        self.nt_fracdep_ionization_ion = np.zeros(np_ * ni)
        self.nt_prob_num_auger = np.zeros(np_ * ni * A1, np.float32)
        self.nt_prob_num_auger[::A1] = 1.
        self.nt_ionenfrac_num_auger = self.nt_prob_num_auger.copy()
        # raw estimators of the transport step
        if est is not None:
            self.J, self.nuJ = est.J.copy(), est.nuJ.copy()
            self.ffheating, self.colheating = est.ffheating.copy(), est.colheating.copy()
            self.bfrate_raw = est.bfrate_raw.copy() if est.nbfcontinua else np.zeros(np_ * nbf)
            self.bin_J_raw, self.bin_nuJ_raw = est.radfield_J.copy(), est.radfield_nuJ.copy()
            self.bin_contribcount = est.radfield_count.copy()
        else:
            raise ValueError("NlteArrays needs the raw estimators of a transport step")
        # outputs
        self.nt_ionization_ratecoeff = np.zeros(np_ * ni)
        self.totalcooling = np.zeros(np_)
        self.cooling_contrib_ion = np.zeros(np_ * ni)
        self.rates = np.zeros(np_ * TE_NRATES)
        self.iters = np.zeros(np_, np.int32)
        ts_start, ts_width, ts_mid, tmin = model_time_grid(m)
        self.params = NlteParams(nts=int(nts), num_lte_timesteps=0, initial_iteration=int(initial_iteration),
                                 nprocs=int(nprocs), nlteiter=30, do_rlc_est=3, deltat=float(ts_width[nts - 1]),
                                 tratmid=float(ts_mid[nts] / tmin), t_mid=float(ts_mid[nts]),
                                 t_current_te=float(ts_mid[nts - 1]), tmin=float(tmin), T_min=float(hdr.mintemp),
                                 T_max=float(hdr.maxtemp), accuracy=1e-3, T_R_min=500., T_R_max=250000.)

    _ARRAYS = {"rho": "rho", "elem_abundance": "elem_abundance", "elem_meanweight": "elem_meanweight",
               "vol_init": "vol_init", "thick": "thick", "deposition_rate_density": "deposition_rate_density",
               "J": "J", "nuJ": "nuJ", "ffheating": "ffheating", "colheating": "colheating",
               "bfrate_raw": "bfrate_raw", "bin_J_raw": "bin_J_raw", "bin_nuJ_raw": "bin_nuJ_raw",
               "bin_contribcount": "bin_contribcount", "TR": "TR", "W": "W", "TJ": "TJ", "Te": "Te", "nne": "nne",
               "nnetot": "nnetot", "groundlevelpop": "groundlevelpop", "partfunct": "partfunct",
               "nlte_pops": "nlte_pops", "bin_TR": "bin_TR", "bin_W": "bin_W", "bfrate_estimator": "bfrate_estimator",
               "nt_frac_heating": "nt_frac_heating", "nt_frac_ionization": "nt_frac_ionization",
               "nt_frac_excitation": "nt_frac_excitation", "nt_nneperion_when_solved": "nt_nneperion_when_solved",
               "nt_timestep_last_solved": "nt_timestep_last_solved", "nt_eff_ionpot": "nt_eff_ionpot",
               "nt_fracdep_ionization_ion": "nt_fracdep_ionization_ion", "nt_prob_num_auger": "nt_prob_num_auger",
               "nt_ionenfrac_num_auger": "nt_ionenfrac_num_auger",
               "nt_ionization_ratecoeff": "nt_ionization_ratecoeff", "totalcooling": "totalcooling",
               "cooling_contrib_ion": "cooling_contrib_ion", "heatingcoolingrates": "rates",
               "nlte_iterations": "iters"}

    def struct(self):
        s = NlteCells()
        s.ncells = len(self.mgi_list)
        s.mgi = self.mgi_list.ctypes.data
        for field, attr in self._ARRAYS.items():
            setattr(s, field, getattr(self, attr).ctypes.data)
        return s

    def copy(self):
        import copy as _c
        o = _c.copy(self)
        for k, v in self.__dict__.items():
            if isinstance(v, np.ndarray):
                setattr(o, k, v.copy())
        o.params = NlteParams.from_buffer_copy(self.params)
        return o

    # the artis_cell_state arrays the next transport step reads (update_grid's outputs)
    _CELLSTATE = [("Te", "Te", C.c_float), ("TR", "TR", C.c_float), ("TJ", "TJ", C.c_float), ("W", "W", C.c_float),
                  ("nne", "nne", C.c_float), ("nnetot", "nnetot", C.c_float),
                  ("groundlevelpop", "groundlevelpop", C.c_float), ("partfunct", "partfunct", C.c_float),
                  ("totalcooling", "totalcooling", C.c_double), ("cooling_contrib_ion", "cooling_contrib_ion", C.c_double),
                  ("nlte_pops", "nlte_pops", C.c_double), ("radfield_bin_TR", "bin_TR", C.c_float),
                  ("radfield_bin_W", "bin_W", C.c_float), ("bfrate_estimator", "bfrate_estimator", C.c_float),
                  ("nt_deposition_rate_density", "deposition_rate_density", C.c_double),
                  ("nt_ionization_ratecoeff", "nt_ionization_ratecoeff", C.c_double),
                  ("nt_prob_num_auger", "nt_prob_num_auger", C.c_float),
                  ("nt_ionenfrac_num_auger", "nt_ionenfrac_num_auger", C.c_float)]

    def apply_to_cellstate(self, model):
        """Write this block's solution into the model's cell state (in place), as update_grid leaves the grid for
        the next update_packets."""
        cs = CellState.from_address(model.cellstate)
        for field, attr, ct in self._CELLSTATE:
            src = getattr(self, attr)
            ptr = getattr(cs, field)
            if not ptr:
                continue
            view = np.ctypeslib.as_array(C.cast(ptr, C.POINTER(ct)), (src.size,))
            view[:] = src
