"""Loader for the CPU oracle (oracle/liboracle.so) -- TEST INFRASTRUCTURE.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this module.
"""
import ctypes as C
import os

import numpy as np

from artis_amd import ffi

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(REPO, "oracle", "liboracle.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            raise RuntimeError(f"{ORACLE_SO} missing: run __graft_entry__.build()")
        L = C.CDLL(ORACLE_SO)
        L.oracle_update_packets.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.POINTER(ffi.RunParams), C.c_int,
                                            C.c_void_p, C.c_int, C.POINTER(ffi.Estimators), C.c_void_p, C.c_int]
        L.oracle_update_packets.restype = C.c_int
        L.oracle_update_packets_g.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.POINTER(ffi.RunParams),
                                              C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.POINTER(ffi.Estimators),
                                              C.c_void_p, C.c_int]
        L.oracle_update_packets_g.restype = C.c_int
        L.oracle_update_packets_v.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.POINTER(ffi.RunParams),
                                              C.c_void_p, C.POINTER(ffi.VpktParams), C.POINTER(ffi.VpktResult),
                                              C.c_int, C.c_void_p, C.c_int, C.POINTER(ffi.Estimators), C.c_void_p,
                                              C.c_int]
        L.oracle_update_packets_v.restype = C.c_int
        L.oracle_qag61_test.argtypes = [C.c_int, C.c_double, C.c_double, C.c_double, C.POINTER(C.c_int),
                                        C.POINTER(C.c_double)]
        L.oracle_qag61_test.restype = C.c_double
        L.oracle_corrphotoioncoeff.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.POINTER(ffi.RunParams)] + \
            [C.c_int] * 5
        L.oracle_corrphotoioncoeff.restype = C.c_double
        _lib = L
    return _lib


def update_packets(model, nts, packets, est=None, nthreads=0, params=None):
    """Run the oracle's update_packets on `packets` (numpy PACKET_DTYPE array, modified in place)."""
    if est is None:
        est = model.new_estimators()
    work = np.zeros(ffi.ARTIS_WORK_COUNT, dtype=np.int64)
    p = params if params is not None else model.params
    rc = lib().oracle_update_packets_g(model.atomic, model.geometry, model.cellstate, C.byref(p),
                                       getattr(model, "gamma_spectra", None), int(nts), packets.ctypes.data,
                                       len(packets), C.byref(est.struct), work.ctypes.data, int(nthreads))
    if rc != 0:
        raise RuntimeError(f"oracle_update_packets -> {rc}")
    return est, work


def update_packets_vpkt(model, nts, packets, vcfg, vout=None, est=None, nthreads=0, params=None):
    """update_packets with VPKT_ON: virtual-packet spectra ADDED into vout (ffi.VpktArrays)."""
    if est is None:
        est = model.new_estimators()
    if vout is None:
        vout = ffi.VpktArrays(vcfg)
    work = np.zeros(ffi.ARTIS_WORK_COUNT, dtype=np.int64)
    p = params if params is not None else model.params
    rc = lib().oracle_update_packets_v(model.atomic, model.geometry, model.cellstate, C.byref(p),
                                       getattr(model, "gamma_spectra", None), C.byref(vcfg.struct),
                                       C.byref(vout.struct), int(nts), packets.ctypes.data, len(packets),
                                       C.byref(est.struct), work.ctypes.data, int(nthreads))
    if rc != 0:
        raise RuntimeError(f"oracle_update_packets_v -> {rc}")
    return est, vout, work


def spectrum(model, packets, nnubins=1000, nprocs=1):
    """Oracle binning of write_partial_lightcurve_spectra (oracle/oracle.cc: oracle_spectrum)."""
    L = lib()
    L.oracle_spectrum.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p,
                                  C.c_void_p]
    L.oracle_spectrum.restype = C.c_int
    nt = model.cfg.ntstep
    spec = np.zeros((nt, nnubins))
    lc = np.zeros(nt)
    lccmf = np.zeros(nt)
    rc = L.oracle_spectrum(model.geometry, packets.ctypes.data, len(packets), nnubins, nprocs, spec.ctypes.data,
                           lc.ctypes.data, lccmf.ctypes.data)
    if rc != 0:
        raise RuntimeError("oracle_spectrum: frequency bin out of range")
    return spec, lc, lccmf


def inverted_lines(model, nts, params=None):
    """(inverted, total): (model cell, line) pairs with a negative Sobolev coefficient (population inversion) under
    the oracle's populations at timestep nts (call model.set_timestep(nts) first)."""
    L = lib()
    L.oracle_inverted_lines.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.POINTER(ffi.RunParams), C.c_int,
                                        C.c_void_p]
    L.oracle_inverted_lines.restype = C.c_int
    out = np.zeros(2, dtype=np.int64)
    p = params if params is not None else model.params
    L.oracle_inverted_lines(model.atomic, model.geometry, model.cellstate, C.byref(p), int(nts), out.ctypes.data)
    return int(out[0]), int(out[1])


def qag61_test(fn, a, b, epsrel):
    """The oracle's gsl_integration_qag(GAUSS61) restatement on closed-form test integrands."""
    st, err = C.c_int(), C.c_double()
    r = lib().oracle_qag61_test(fn, a, b, epsrel, C.byref(st), C.byref(err))
    return r, st.value, err.value


def corrphotoioncoeff(model, nts, mgi, ul, t, brute=False, params=None):
    """get_corrphotoioncoeff as the oracle's macro-atom sees it.  brute=1: dense Gauss-Legendre quadrature of the
    same integrand; brute=2: the same qag restatement at epsrel 1e-10 (the reference runs it at 1e-3)."""
    p = params if params is not None else model.params
    r = lib().oracle_corrphotoioncoeff(model.atomic, model.geometry, model.cellstate, C.byref(p),
                                       int(nts), int(mgi), int(ul), int(t), int(brute))
    if not np.isfinite(r):
        raise ValueError(f"oracle_corrphotoioncoeff(mgi={mgi}, level={ul}, target={t}): no photoionisation target "
                         f"or a non-finite integral")
    return r


def ionising_levels(model):
    """Unique indices of every level with photoionisation targets (level < ionisinglevels of a non-top ion)."""
    class Hdr(C.Structure):  # leading fields of artis_atomic_tables (include/artis_gpu.h)
        _fields_ = ffi.AtomicHeader._fields_ + [("ion_ionstage", C.c_void_p), ("ion_nlevels", C.c_void_p),
                                                ("ion_uniqueleveloffset", C.c_void_p),
                                                ("ion_ionisinglevels", C.c_void_p)]

    hdr = Hdr.from_address(model.atomic)
    n = lambda p, k: np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_int32)), (k,))  # noqa: E731
    nions = n(hdr.elem_nions, model.nelements)
    ionoff = n(hdr.elem_uniqueionoffset, model.nelements)
    lvoff = n(hdr.ion_uniqueleveloffset, model.nions_total)
    nion = n(hdr.ion_ionisinglevels, model.nions_total)
    out = []
    for e in range(model.nelements):
        for i in range(nions[e] - 1):
            ui = ionoff[e] + i
            out += list(range(lvoff[ui], lvoff[ui] + nion[ui]))
    return out


def spectra(model, packets, nnubins=1000, nprocs=1, abin=-1, syn_dir=(0., 0., 1.), emission_res=True, stokes=False):
    """The oracle's exspec binning (oracle_spectra: add_to_spec_res / add_to_lc_res in packet order)."""
    L = lib()
    L.oracle_spectra.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.POINTER(ffi.SpectraRequest),
                                 C.POINTER(ffi.SpectraOut)]
    L.oracle_spectra.restype = C.c_int
    out = ffi.SpectraArrays(model.cfg.ntstep, nnubins, model.nelements, model.maxnions, emission_res, stokes)
    req = ffi.spectra_request(nnubins, nprocs, abin, syn_dir)
    rc = L.oracle_spectra(model.atomic, model.geometry, packets.ctypes.data, len(packets), C.byref(req),
                          C.byref(out.struct))
    if rc != 0:
        raise RuntimeError(f"oracle_spectra -> {rc}")
    return out


def solve_temperatures(model, te, params=None, nthreads=0):
    """oracle_solve_temperatures on a TeArrays block (in place); returns the status."""
    L = lib()
    L.oracle_solve_temperatures.argtypes = [C.c_void_p, C.POINTER(ffi.RunParams), C.c_void_p,
                                            C.POINTER(ffi.TeParams), C.POINTER(ffi.TeCells), C.c_int, C.c_int]
    s = te.struct()
    rc = L.oracle_solve_temperatures(model.atomic, C.byref(params if params is not None else model.params), te.tables,
                                     C.byref(te.params), C.byref(s), model.npts_model, nthreads)
    return rc


def prepare_temperatures(model, te, prep, params=None, nthreads=0):
    """oracle_prepare_temperatures on a TeArrays + UgArrays pair (fills prep's outputs); returns the status."""
    L = lib()
    L.oracle_prepare_temperatures.argtypes = [C.c_void_p, C.POINTER(ffi.RunParams), C.c_void_p,
                                              C.POINTER(ffi.TeParams), C.POINTER(ffi.UgPrepare),
                                              C.POINTER(ffi.TeCells), C.c_int, C.c_int]
    s = te.struct()
    p = prep.struct()
    return L.oracle_prepare_temperatures(model.atomic, C.byref(params if params is not None else model.params),
                                         te.tables, C.byref(te.params), C.byref(p), C.byref(s), model.npts_model,
                                         nthreads)


def update_grid_nlte(model, nt, arr, params=None, nthreads=0):
    """oracle_update_grid_nlte on an NlteArrays block (in place) with an NtDataHandle; returns the status."""
    L = lib()
    L.oracle_update_grid_nlte.argtypes = [C.c_void_p, C.POINTER(ffi.RunParams), C.POINTER(ffi.NtShells),
                                          C.POINTER(ffi.NlteParams), C.POINTER(ffi.NlteCells), C.c_int, C.c_int]
    s = arr.struct()
    return L.oracle_update_grid_nlte(model.atomic, C.byref(params if params is not None else model.params),
                                     C.byref(nt.shells), C.byref(arr.params), C.byref(s), model.npts_model, nthreads)
