"""Packet / estimator comparison helpers shared by the GPU parity tests, the golden tests and smoke().

Integer, enum and index fields of the 304-byte record must be identical.  Floating-point fields are compared
with a relative tolerance of FP_RTOL: the engine evaluates the same double-precision expressions in the same
order as the oracle (both built with -ffp-contract=off), but the device libm (exp/log/pow/sqrt of ROCm's ocml)
and glibc may differ in the last ulp, and a few hundred events per packet compound that to ~1e-14.
Estimators are float64 sums accumulated with atomics in a schedule-dependent order: ESTIMATOR_RTOL.
"""
import numpy as np

FP_RTOL = 1e-9
# stats of the reference's per-OpenMP-thread cellhistory cache (CTR_UPDATECELL, CTR_COOLINGRATECALCCOUNTER,
# stats.h): the engine has no per-thread cache (per-cell tables in HBM instead), so these are not compared
CACHE_COUNTERS = [31, 32]
# CTR_UPSCATTER / CTR_DOWNSCATTER compare nu_cmf after an electron scattering with nu_cmf before
# (rpkt.cc escat branch); the comoving frequency is unchanged by Thomson scattering up to the rounding of the
# frame transforms, so the split is decided by last-ulp noise.  Only their sum is an event count.
ROUNDING_SPLIT_COUNTERS = (29, 30)
ESTIMATOR_RTOL = 1e-9

INT_FIELDS = ["where", "type", "last_cross", "interactions", "nscatterings", "last_event", "next_trans",
              "emissiontype", "absorptiontype", "trueemissiontype", "escape_type", "scat_count", "number",
              "originated_from_particlenotgamma", "pellet_decaytype", "pellet_nucindex", "mastate"]
FP_FIELDS = ["pos", "dir", "e_cmf", "e_rf", "nu_cmf", "nu_rf", "em_pos", "em_time", "prop_time", "trueem_time",
             "absorptionfreq", "absorptiondir", "stokes", "pol_dir", "tdecay", "escape_time",
             "trueemissionvelocity"]


def discrete_mismatch(a, b):
    """Boolean mask of packets whose integer/enum/index state differs."""
    bad = np.zeros(len(a), dtype=bool)
    for f in INT_FIELDS:
        x, y = a[f], b[f]
        if x.dtype.names:  # mastate
            for sub in x.dtype.names:
                bad |= x[sub] != y[sub]
        else:
            bad |= (x != y).reshape(len(a), -1).any(axis=1)
    return bad


def fp_max_rel(a, b, mask=None):
    """max over FP fields of |a-b| / max(|b|, tiny) on the packets selected by mask."""
    out = {}
    sel = np.ones(len(a), dtype=bool) if mask is None else mask
    for f in FP_FIELDS:
        x = a[f][sel].astype(np.float64)
        y = b[f][sel].astype(np.float64)
        scale = np.maximum(np.abs(y), 1e-300)
        d = np.abs(x - y)
        # vectors: compare against the vector norm (a component can pass through zero)
        if x.ndim == 2:
            scale = np.maximum(np.linalg.norm(y, axis=1, keepdims=True), 1e-300)
        out[f] = float((d / scale).max()) if d.size else 0.0
    return out


def assert_packets_match(gpu, ref, max_discrete_mismatch=0, rtol=FP_RTOL):
    bad = discrete_mismatch(gpu, ref)
    assert bad.sum() <= max_discrete_mismatch, f"{int(bad.sum())} of {len(gpu)} packets differ in discrete state"
    rel = fp_max_rel(gpu, ref, ~bad)
    worst = max(rel.values()) if rel else 0.0
    assert worst <= rtol, rel
    return int(bad.sum()), worst


def spectrum(packets, nbins=1000, nu_min=1e14, nu_max=5e15):
    """Energy of escaped packets binned in log nu_rf (spec.out binning over [NU_MIN_R, NU_MAX_R], spectrum.cc:339-362)."""
    esc = packets["type"] == 32
    nu = packets["nu_rf"][esc]
    e = packets["e_rf"][esc]
    edges = np.exp(np.linspace(np.log(nu_min), np.log(nu_max), nbins + 1))
    h, _ = np.histogram(nu, bins=edges, weights=e)
    return h


def spectrum_l1(a, b):
    sa, sb = spectrum(a), spectrum(b)
    return float(np.abs(sa - sb).sum() / max(np.abs(sb).sum(), 1e-300))


def counters_equal(a, b):
    a, b = np.asarray(a), np.asarray(b)
    keep = np.ones(len(a), dtype=bool)
    keep[CACHE_COUNTERS] = False
    keep[list(ROUNDING_SPLIT_COUNTERS)] = False
    up, down = ROUNDING_SPLIT_COUNTERS
    return bool((a[keep] == b[keep]).all() and a[up] + a[down] == b[up] + b[down])


def assert_estimators_match(eg, eo, exact_counts=True, rtol=ESTIMATOR_RTOL):
    for name in ("J", "nuJ", "ffheating", "colheating", "gamma", "bfheating", "rpkt_emiss"):
        x, y = getattr(eg, name), getattr(eo, name)
        scale = max(np.abs(y).max(), 1e-300) if y.size else 1e-300
        assert np.abs(x - y).max(initial=0.0) <= rtol * scale, (name, np.abs(x - y).max() / scale)
    # time_step[nts] scalars (globals.h:20-40) and nt_energy_deposited
    for name in ("cmf_lum", "gamma_dep", "positron_dep", "electron_dep", "electron_emission", "alpha_dep",
                 "alpha_emission", "gamma_emission", "nt_energy_deposited"):
        x, y = getattr(eg.struct, name), getattr(eo.struct, name)
        assert abs(x - y) <= rtol * max(abs(y), 1e-300), (name, x, y)
    # nebular estimators (DETAILED_BF_ESTIMATORS_ON / MULTIBIN_RADFIELD_MODEL_ON); bin contribution counts exact
    for name in ("bfrate_raw", "radfield_J", "radfield_nuJ"):
        x, y = getattr(eg, name, np.zeros(0)), getattr(eo, name, np.zeros(0))
        assert x.shape == y.shape, name
        if y.size:
            scale = max(np.abs(y).max(), 1e-300)
            assert np.abs(x - y).max() <= rtol * scale, (name, np.abs(x - y).max() / scale)
    # Compton / pair-production emissivities (float, as globals::compton_emiss): float rounding of the sums
    x, y = getattr(eg, "compton_emiss", np.zeros(0)), getattr(eo, "compton_emiss", np.zeros(0))
    if y.size and np.abs(y).max() > 0:
        scale = float(np.abs(y).max())
        assert np.abs(x.astype(np.float64) - y).max() <= max(rtol, 2e-6) * scale, (
            "compton_emiss", np.abs(x.astype(np.float64) - y).max() / scale)
    if exact_counts and getattr(eo, "radfield_count", np.zeros(0)).size:
        assert np.array_equal(eg.radfield_count, eo.radfield_count)
    if exact_counts:
        assert eg.struct.nesc == eo.struct.nesc
        assert eg.struct.pellet_decays == eo.struct.pellet_decays
        assert counters_equal(eg.counters, eo.counters), (eg.counters, eo.counters)
        assert (eg.ecounter == eo.ecounter).all()
        assert (eg.acounter == eo.acounter).all()
