"""ctypes mirrors of the C-ABI structs in include/artis_gpu.h and model_synth.h.

Plain data plumbing: every struct here has the same field order and types as the C header, and
tests/test_abi.py checks sizes/offsets against the compiled libraries.
"""
import ctypes as C

import numpy as np

ARTIS_WORK_COUNT = 16
ARTIS_COUNTER_COUNT = 34

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
    ]


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

    def __init__(self, npts_model, nelements, maxnions, nlines):
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
