"""Synthetic ARTIS model (atomic data + grid + LTE cell state + initial r-packets) via libartis_model.so.

Input generation for tests and bench only (the reference's input()/grid_init()/update_grid() stand-in,
SURVEY.md §8(d)); the engine itself is in libartis_gpu.so.
"""
import ctypes as C
import os

import numpy as np

from . import ffi

_LIBDIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib")
_model_lib = None


def model_lib():
    global _model_lib
    if _model_lib is None:
        path = os.path.join(_LIBDIR, "libartis_model.so")
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: run __graft_entry__.build() first")
        lib = C.CDLL(path)
        lib.artis_synth_default_config.argtypes = [C.POINTER(ffi.SynthConfig)]
        lib.artis_model_synth.argtypes = [C.POINTER(ffi.SynthConfig)]
        lib.artis_model_synth.restype = C.c_void_p
        lib.artis_model_from_files.argtypes = [C.POINTER(ffi.SynthConfig), C.c_char_p, C.c_char_p, C.c_char_p]
        lib.artis_model_from_files.restype = C.c_void_p
        lib.artis_model_free.argtypes = [C.c_void_p]
        for fn in ("artis_model_atomic", "artis_model_geometry", "artis_model_cellstate", "artis_model_te_tables"):
            getattr(lib, fn).argtypes = [C.c_void_p]
            getattr(lib, fn).restype = C.c_void_p
        lib.artis_model_run_params.argtypes = [C.c_void_p, C.POINTER(ffi.RunParams)]
        lib.artis_model_set_timestep.argtypes = [C.c_void_p, C.c_int]
        lib.artis_model_advance.argtypes = [C.c_void_p, C.c_int]
        lib.artis_model_init_rpackets.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_uint64, C.c_double, C.c_void_p]
        lib.artis_model_set_gamma_lines.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_void_p]
        lib.artis_model_gamma_spectra.argtypes = [C.c_void_p]
        lib.artis_model_gamma_spectra.restype = C.c_void_p
        lib.artis_model_init_pellets.argtypes = [C.c_void_p, C.c_int, C.c_uint64, C.c_double, C.c_double, C.c_double,
                                                 C.c_void_p]
        lib.artis_model_config.argtypes = [C.c_void_p, C.POINTER(ffi.SynthConfig)]
        lib.artis_model_npts_model.argtypes = [C.c_void_p]
        lib.artis_model_npts_model.restype = C.c_int64
        lib.artis_model_radfield_nbins.argtypes = [C.c_void_p]
        lib.artis_model_total_nlte_levels.argtypes = [C.c_void_p]
        lib.artis_model_ion_ionstage.argtypes = [C.c_void_p]
        lib.artis_model_ion_ionstage.restype = C.c_void_p
        lib.artis_model_ion_ground_statweight.argtypes = [C.c_void_p, C.c_void_p]
        lib.artis_model_ion_ground_statweight.restype = None
        _model_lib = lib
    return _model_lib


def default_config(**overrides):
    cfg = ffi.SynthConfig()
    model_lib().artis_synth_default_config(C.byref(cfg))
    for k, v in overrides.items():
        setattr(cfg, k, v)
    return cfg


class Model:
    """Owns one model; exposes the raw C struct pointers for the engine and the oracle.

    Synthetic by default; with files=(input.txt, model.txt, abundances.txt) the run
    parameters, time grid, ejecta model and abundances come from the reference's own input files
    (artis_model_from_files), with synthetic atomic data.  A model.txt.xz is decompressed next to a temp copy.
    """

    def __init__(self, cfg=None, files=None, **overrides):
        self.cfg = cfg if cfg is not None else default_config(**overrides)
        self._lib = model_lib()
        self._tmp = None
        if files is not None:
            inp, mod, ab = (os.fspath(f) for f in files)
            if mod.endswith(".xz"):
                import lzma
                import tempfile

                self._tmp = tempfile.TemporaryDirectory()
                plain = os.path.join(self._tmp.name, "model.txt")
                with lzma.open(mod, "rb") as fin, open(plain, "wb") as fout:
                    fout.write(fin.read())
                mod = plain
            self._h = self._lib.artis_model_from_files(C.byref(self.cfg), inp.encode(), mod.encode(), ab.encode())
            if not self._h:
                raise RuntimeError(f"artis_model_from_files({inp}, {mod}, {ab}) failed")
            # the C side adopted ntstep / times / seed from input.txt: mirror them in self.cfg
            self._lib.artis_model_config(self._h, C.byref(self.cfg))
        else:
            self._h = self._lib.artis_model_synth(C.byref(self.cfg))
        if not self._h:
            raise RuntimeError("artis_model_synth failed")
        self.atomic = self._lib.artis_model_atomic(self._h)
        self.geometry = self._lib.artis_model_geometry(self._h)
        self.cellstate = self._lib.artis_model_cellstate(self._h)
        self.params = ffi.RunParams()
        self._lib.artis_model_run_params(self._h, C.byref(self.params))
        self.npts_model = int(self._lib.artis_model_npts_model(self._h))
        # a few counts straight from the atomic-table header (first 8 int32 of artis_atomic_tables)
        hdr = (C.c_int32 * 8).from_address(self.atomic)
        (self.nelements, self.maxnions, self.nions_total, self.nlevels_total, self.nlines,
         self.nbfcontinua, self.nbfcontinua_ground, self.ncoolingterms) = list(hdr)
        self.nts = 0
        self._load_gamma_lines()
        self.gamma_spectra = self._lib.artis_model_gamma_spectra(self._h)

    # the reference's own gamma-line data files (data/ni56_lines.txt, data/co56_lines.txt), package data
    GAMMA_LINE_FILES = {0: "ni56_lines.txt", 1: "co56_lines.txt"}

    def _load_gamma_lines(self):
        d = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "gamma_lines")
        for nuc, fn in self.GAMMA_LINE_FILES.items():
            path = os.path.join(d, fn)
            if not os.path.exists(path):
                continue
            with open(path) as f:  # read_gamma_spectrum (gammapkt.cc:58-89): count, then "E[MeV] prob" rows
                tok = f.read().split()
            n = int(tok[0])
            vals = np.array([float(x) for x in tok[1:1 + 2 * n]]).reshape(n, 2)
            en = np.ascontiguousarray(vals[:, 0])
            pr = np.ascontiguousarray(vals[:, 1])
            rc = self._lib.artis_model_set_gamma_lines(self._h, nuc, n, en.ctypes.data, pr.ctypes.data)
            if rc != 0:
                raise RuntimeError(f"artis_model_set_gamma_lines({nuc}) -> {rc}")

    def set_timestep(self, nts):
        rc = self._lib.artis_model_set_timestep(self._h, int(nts))
        if rc != 0:
            raise RuntimeError(f"artis_model_set_timestep({nts}) -> {rc}")
        self.nts = nts

    def advance(self, nts):
        """update_grid's host bookkeeping for timestep nts (rho(t), grey opacity, thick flag), leaving temperatures,
        populations and cooling as they are (the timestep loop writes them from the GPU solution)."""
        rc = self._lib.artis_model_advance(self._h, int(nts))
        if rc != 0:
            raise RuntimeError(f"artis_model_advance({nts}) -> {rc}")
        self.nts = nts

    def init_rpackets(self, nts, npkts, seed=1, etot=1e45):
        pk = np.zeros(npkts, dtype=ffi.PACKET_DTYPE)
        rc = self._lib.artis_model_init_rpackets(self._h, int(nts), int(npkts), C.c_uint64(seed), float(etot),
                                                 pk.ctypes.data)
        if rc != 0:
            raise RuntimeError(f"artis_model_init_rpackets -> {rc}")
        return pk

    def init_pellets(self, npkts, seed=1, etot=1e45, t_model_days=None, frac_initial=0.02):
        """Radioactive pellets at tmin (packet_init stand-in, see model_synth.h)."""
        if t_model_days is None:
            t_model_days = 0.5 * self.cfg.tmin_days
        pk = np.zeros(npkts, dtype=ffi.PACKET_DTYPE)
        rc = self._lib.artis_model_init_pellets(self._h, int(npkts), C.c_uint64(seed), float(etot),
                                                float(t_model_days), float(frac_initial), pk.ctypes.data)
        if rc != 0:
            raise RuntimeError(f"artis_model_init_pellets -> {rc}")
        return pk

    def new_estimators(self):
        p = self.params
        return ffi.EstimatorArrays(self.npts_model, self.nelements, self.maxnions, self.nlines,
                                   self.nbfcontinua if p.detailed_bf_estimators else 0,
                                   self.radfield_nbins if p.multibin_radfield else 0)

    @property
    def radfield_nbins(self):
        return int(self._lib.artis_model_radfield_nbins(self._h))

    @property
    def total_nlte_levels(self):
        return int(self._lib.artis_model_total_nlte_levels(self._h))

    def ion_ionstage(self):
        p = self._lib.artis_model_ion_ionstage(self._h)
        return np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_int32)), (self.nions_total,)).copy()

    def ion_ground_statweight(self):
        g = np.zeros(self.nions_total, dtype=np.float32)
        self._lib.artis_model_ion_ground_statweight(self._h, g.ctypes.data)
        return g

    def ion_element(self):
        """element index of every unique ion"""
        hdr = ffi.AtomicHeader.from_address(self.atomic)
        nions = np.ctypeslib.as_array(C.cast(hdr.elem_nions, C.POINTER(C.c_int32)), (self.nelements,))
        return np.repeat(np.arange(self.nelements), nions)

    def close(self):
        if self._h:
            self._lib.artis_model_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
