"""artis_amd -- MI355X-native packet-propagation engine for ARTIS (update_packets hot path).

The product is the C-ABI library artis_amd/lib/libartis_gpu.so (include/artis_gpu.h): hand-written HIP
kernels for gfx950.  This module is a thin ctypes mirror of that ABI for tests, the bench and the
multi-GPU driver.  There is no CPU fallback: if the library or a GPU is missing, Engine() raises.
"""
import ctypes as C
import os

import numpy as np

from . import ffi

_LIBDIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib")
GPU_SO = os.path.join(_LIBDIR, "libartis_gpu.so")
# diagnostics only: load an alternative build of the same engine (e.g. the in-kernel timestamp variant)
_GPU_SO_LOAD = os.environ.get("ARTIS_GPU_SO", GPU_SO)

# every function declared in include/artis_gpu.h (tests/test_abi.py checks they are exported)
ABI_SYMBOLS = [
    "artis_gpu_init", "artis_gpu_init_gamma", "artis_gpu_finalize", "artis_gpu_upload_cellstate", "artis_gpu_update_packets",
    "artis_gpu_packets_upload", "artis_gpu_packets_download", "artis_gpu_packets_snapshot",
    "artis_gpu_packets_restore", "artis_gpu_update_packets_resident", "artis_gpu_estimators_zero",
    "artis_gpu_estimators_download", "artis_gpu_estimator_block_doubles", "artis_gpu_estimator_block_to_device",
    "artis_gpu_estimator_block_from_device", "artis_gpu_last_transport_ms", "artis_gpu_last_precompute_ms",
    "artis_gpu_last_work_counts", "artis_gpu_last_rounds", "artis_gpu_spectrum", "artis_gpu_spectra", "artis_gpu_last_kernel_times",
    "artis_gpu_last_kernel_class_times", "artis_gpu_last_error", "artis_gpu_abi_version",
    "artis_gpu_vpkt_init", "artis_gpu_vpkt_zero", "artis_gpu_vpkt_download", "artis_gpu_vpkt_last_stats", "artis_gpu_vpkt_last_work",
    "artis_estimator_block_len", "artis_estimator_block_pack", "artis_estimator_block_unpack",
    "artis_estimator_block_average_scalars",
    "artis_gpu_comm_unique_id", "artis_gpu_comm_init", "artis_gpu_estimators_allreduce", "artis_gpu_comm_finalize",
    "artis_gpu_solve_temperatures", "artis_gpu_last_te_ms", "artis_gpu_prepare_temperatures",
    "artis_gpu_update_grid_nlte", "artis_gpu_last_nlte_ms", "artis_gpu_table_info", "artis_gpu_vpkt_last_drains",
]

_gpu_lib = None


def engine_src_sha():
    """sha256 (16 hex) of the engine's sources (artis_amd/csrc/engine/*, include/*.h): keys committed profiles
    (profiles/pmc_*.json) to the code they measured -- the GPU box gets the tree without .git."""
    import hashlib

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    h = hashlib.sha256()
    for d in (os.path.join(repo, "artis_amd", "csrc", "engine"), os.path.join(repo, "include")):
        for f in sorted(os.listdir(d)):
            if f.endswith((".hip", ".h")):
                h.update(f.encode())
                with open(os.path.join(d, f), "rb") as fh:
                    h.update(fh.read())
    return h.hexdigest()[:16]


def gpu_lib():
    """Load libartis_gpu.so (fails loudly if it was not built)."""
    global _gpu_lib
    if _gpu_lib is None:
        if not os.path.exists(_GPU_SO_LOAD):
            raise RuntimeError(f"{_GPU_SO_LOAD} missing: the HIP engine was not built (run __graft_entry__.build())")
        L = C.CDLL(_GPU_SO_LOAD)
        vp = C.c_void_p
        L.artis_gpu_init.argtypes = [C.c_int, vp, vp, C.POINTER(ffi.RunParams)]
        L.artis_gpu_init_gamma.argtypes = [vp]
        L.artis_gpu_upload_cellstate.argtypes = [C.c_int, vp]
        L.artis_gpu_update_packets.argtypes = [C.c_int, C.c_int, vp, C.c_int, C.POINTER(ffi.Estimators)]
        L.artis_gpu_packets_upload.argtypes = [vp, C.c_int]
        L.artis_gpu_packets_download.argtypes = [vp, C.c_int]
        L.artis_gpu_update_packets_resident.argtypes = [C.c_int, C.c_int]
        L.artis_gpu_estimators_download.argtypes = [C.POINTER(ffi.Estimators)]
        L.artis_gpu_estimator_block_doubles.restype = C.c_size_t
        L.artis_gpu_estimator_block_to_device.argtypes = [vp]
        L.artis_gpu_estimator_block_from_device.argtypes = [vp]
        L.artis_gpu_last_transport_ms.restype = C.c_double
        L.artis_gpu_last_precompute_ms.restype = C.c_double
        L.artis_gpu_last_work_counts.argtypes = [vp]
        L.artis_gpu_table_info.argtypes = [vp]
        L.artis_gpu_vpkt_last_drains.restype = C.c_int64
        L.artis_gpu_last_error.restype = C.c_char_p
        L.artis_gpu_last_rounds.restype = C.c_int64
        L.artis_gpu_spectrum.argtypes = [C.c_int, C.c_int, vp, vp, vp]
        L.artis_gpu_spectra.argtypes = [C.POINTER(ffi.SpectraRequest), C.POINTER(ffi.SpectraOut)]
        L.artis_gpu_vpkt_init.argtypes = [C.POINTER(ffi.VpktParams)]
        L.artis_gpu_vpkt_download.argtypes = [C.POINTER(ffi.VpktResult), C.c_int]
        L.artis_gpu_vpkt_last_stats.argtypes = [C.POINTER(C.c_double), C.POINTER(C.c_int64), C.POINTER(C.c_int64)]
        L.artis_gpu_vpkt_last_work.argtypes = [C.POINTER(C.c_int64)]
        L.artis_estimator_block_len.argtypes = [C.c_int] * 6
        L.artis_estimator_block_len.restype = C.c_size_t
        L.artis_estimator_block_pack.argtypes = [C.POINTER(ffi.Estimators)] + [C.c_int] * 6 + [vp]
        L.artis_estimator_block_unpack.argtypes = [vp] + [C.c_int] * 6 + [C.POINTER(ffi.Estimators)]
        L.artis_estimator_block_average_scalars.argtypes = [vp] + [C.c_int] * 4
        L.artis_gpu_comm_unique_id.argtypes = [vp]
        L.artis_gpu_comm_init.argtypes = [C.c_int, C.c_int, vp]
        L.artis_gpu_comm_finalize.restype = None
        L.artis_gpu_solve_temperatures.argtypes = [vp, C.POINTER(ffi.TeParams), C.POINTER(ffi.TeCells)]
        L.artis_gpu_last_te_ms.restype = C.c_double
        L.artis_gpu_prepare_temperatures.argtypes = [vp, C.POINTER(ffi.TeParams), C.POINTER(ffi.UgPrepare),
                                                     C.POINTER(ffi.TeCells)]
        L.artis_gpu_update_grid_nlte.argtypes = [C.POINTER(ffi.NtShells), C.POINTER(ffi.NlteParams),
                                                 C.POINTER(ffi.NlteCells)]
        L.artis_gpu_last_nlte_ms.restype = C.c_double
        _gpu_lib = L
    return _gpu_lib


class EngineError(RuntimeError):
    pass


def comm_unique_id():
    """ncclGetUniqueId on this process (rank 0), as bytes to hand to every rank."""
    buf = C.create_string_buffer(ffi.COMM_ID_BYTES)
    rc = gpu_lib().artis_gpu_comm_unique_id(buf)
    if rc != 0:
        raise EngineError(f"artis_gpu_comm_unique_id -> {rc}: {gpu_lib().artis_gpu_last_error().decode()}")
    return buf.raw


class Engine:
    """One HIP device's engine instance bound to a model (atomic tables + geometry)."""

    def __init__(self, model, device=0, params=None):
        self.lib = gpu_lib()
        self.model = model
        self.params = params if params is not None else model.params
        self._check(self.lib.artis_gpu_init(int(device), model.atomic, model.geometry, C.byref(self.params)), "init")
        if getattr(model, "gamma_spectra", None):
            self._check(self.lib.artis_gpu_init_gamma(model.gamma_spectra), "init_gamma")
        self.cell_nts = None

    def _check(self, rc, what):
        if rc != 0:
            msg = self.lib.artis_gpu_last_error()
            raise EngineError(f"artis_gpu_{what} -> {rc}: {msg.decode() if msg else ''}")

    def solve_temperatures(self, te):
        """update_grid's temperature / ionisation solution (artis_gpu_solve_temperatures) on a TeArrays block, in
        place; returns the device milliseconds."""
        s = te.struct()
        self._check(self.lib.artis_gpu_solve_temperatures(te.tables, C.byref(te.params), C.byref(s)),
                    "solve_temperatures")
        return float(self.lib.artis_gpu_last_te_ms())

    def prepare_temperatures(self, te, prep):
        """update_grid_cell's estimator preparation (artis_gpu_prepare_temperatures) for the cells of a TeArrays
        block from the raw estimators in a UgArrays block; fills prep's outputs."""
        s = te.struct()
        self._check(self.lib.artis_gpu_prepare_temperatures(te.tables, C.byref(te.params), C.byref(prep.struct()),
                                                            C.byref(s)), "prepare_temperatures")

    def update_grid_nlte(self, nt, arr):
        """update_grid for the nebular options (artis_gpu_update_grid_nlte) on an NlteArrays block, in place; nt: an
        NtDataHandle (the Spencer-Fano shells) or None.  Returns the device milliseconds."""
        s = arr.struct()
        self._check(self.lib.artis_gpu_update_grid_nlte(C.byref(nt.shells) if nt is not None else None,
                                                        C.byref(arr.params), C.byref(s)), "update_grid_nlte")
        return float(self.lib.artis_gpu_last_nlte_ms())

    def upload_cellstate(self, nts):
        self._check(self.lib.artis_gpu_upload_cellstate(int(nts), self.model.cellstate), "upload_cellstate")
        self.cell_nts = nts

    def update_packets(self, nts, packets, est=None, my_rank=None):
        """Drop-in update_packets(my_rank, nts, packets): packets modified in place, estimators added to est."""
        if est is None:
            est = self.model.new_estimators()
        rank = self.params.rank if my_rank is None else my_rank
        self._check(self.lib.artis_gpu_update_packets(int(rank), int(nts), packets.ctypes.data, len(packets),
                                                      C.byref(est.struct)), "update_packets")
        return est

    # device-resident path
    def upload(self, packets):
        self._check(self.lib.artis_gpu_packets_upload(packets.ctypes.data, len(packets)), "packets_upload")
        self.npkts = len(packets)

    def download(self, packets):
        self._check(self.lib.artis_gpu_packets_download(packets.ctypes.data, len(packets)), "packets_download")

    def snapshot(self):
        self._check(self.lib.artis_gpu_packets_snapshot(), "packets_snapshot")

    def restore(self):
        self._check(self.lib.artis_gpu_packets_restore(), "packets_restore")

    def zero_estimators(self):
        self._check(self.lib.artis_gpu_estimators_zero(), "estimators_zero")

    def step_resident(self, nts, my_rank=None):
        rank = self.params.rank if my_rank is None else my_rank
        self._check(self.lib.artis_gpu_update_packets_resident(int(rank), int(nts)), "update_packets_resident")

    def download_estimators(self, est=None):
        if est is None:
            est = self.model.new_estimators()
        self._check(self.lib.artis_gpu_estimators_download(C.byref(est.struct)), "estimators_download")
        return est

    def estimator_block_doubles(self):
        return int(self.lib.artis_gpu_estimator_block_doubles())

    def estimator_block_to_device(self, dptr):
        self._check(self.lib.artis_gpu_estimator_block_to_device(C.c_void_p(dptr)), "estimator_block_to_device")

    def estimator_block_from_device(self, dptr):
        self._check(self.lib.artis_gpu_estimator_block_from_device(C.c_void_p(dptr)), "estimator_block_from_device")

    def last_transport_ms(self):
        return float(self.lib.artis_gpu_last_transport_ms())

    def last_precompute_ms(self):
        return float(self.lib.artis_gpu_last_precompute_ms())

    def last_work(self):
        w = np.zeros(ffi.ARTIS_WORK_COUNT, dtype=np.int64)
        self.lib.artis_gpu_last_work_counts(w.ctypes.data)
        return w

    def table_info(self):
        """Per-cell table coverage: {"cells", "linecoef_rows", "linecoef_bytes", "macache_rows", "macache_bytes",
        "marates_bytes"} (artis_gpu_table_info)."""
        w = np.zeros(11, dtype=np.int64)
        self._check(self.lib.artis_gpu_table_info(w.ctypes.data), "table_info")
        return dict(zip(("cells", "linecoef_rows", "linecoef_bytes", "macache_rows", "macache_bytes",
                         "marates_bytes", "ma_jumps_recorded", "ma_jumps", "ma_level_records",
                         "ma_level_bytes", "ma_pool_bytes"), (int(x) for x in w)))

    def spectrum(self, nnubins=1000, nprocs=1):
        """Device-binned spectrum [ntstep, nnubins] and light curves (lum, lumcmf) of the resident packets."""
        nt = self.model.cfg.ntstep
        spec = np.zeros((nt, nnubins))
        lc = np.zeros(nt)
        lccmf = np.zeros(nt)
        self._check(self.lib.artis_gpu_spectrum(int(nnubins), int(nprocs), spec.ctypes.data, lc.ctypes.data,
                                                lccmf.ctypes.data), "spectrum")
        return spec, lc, lccmf

    def spectra(self, nnubins=1000, nprocs=1, abin=-1, syn_dir=(0., 0., 1.), emission_res=True, stokes=False,
                out=None):
        """exspec spectra of the resident packets (artis_gpu_spectra): ADDED into out (ffi.SpectraArrays)."""
        if out is None:
            out = ffi.SpectraArrays(self.model.cfg.ntstep, nnubins, self.model.nelements, self.model.maxnions,
                                    emission_res, stokes)
        req = ffi.spectra_request(nnubins, nprocs, abin, syn_dir)
        self._check(self.lib.artis_gpu_spectra(C.byref(req), C.byref(out.struct)), "spectra")
        return out

    # virtual packets (VPKT_ON)
    def vpkt_init(self, cfg):
        """Switch virtual packets on (cfg: ffi.VpktConfig); accumulators start at zero."""
        self._vpkt_cfg = cfg
        self._check(self.lib.artis_gpu_vpkt_init(C.byref(cfg.struct)), "vpkt_init")

    def vpkt_zero(self):
        self._check(self.lib.artis_gpu_vpkt_zero(), "vpkt_zero")

    def vpkt_download(self, out=None, reset_counters=False):
        """ADD the device virtual-packet spectra / grid / counters into out (ffi.VpktArrays)."""
        if out is None:
            out = ffi.VpktArrays(self._vpkt_cfg)
        self._check(self.lib.artis_gpu_vpkt_download(C.byref(out.struct), int(bool(reset_counters))), "vpkt_download")
        return out

    def vpkt_last_stats(self):
        """(ms of the k_vpkt launches, spawn records, traced virtual packets) of the last update."""
        ms = C.c_double()
        sp = C.c_int64()
        tr = C.c_int64()
        self.lib.artis_gpu_vpkt_last_stats(C.byref(ms), C.byref(sp), C.byref(tr))
        return ms.value, sp.value, tr.value

    def vpkt_last_drains(self):
        """Launches of the last update resumed after the virtual-packet spawn buffer filled."""
        return int(self.lib.artis_gpu_vpkt_last_drains())

    def vpkt_last_work(self):
        """{segments, lines, bf_active, escaped} of the last update's virtual packets."""
        w = (C.c_int64 * 4)()
        self.lib.artis_gpu_vpkt_last_work(w)
        return dict(zip(("segments", "lines", "bf_active", "escaped"), (int(x) for x in w)))

    def last_kernel_times(self):
        """{class: (ms, launches)} for the last transport: rpkt (k_rpkt), ma (k_ma), kpkt (k_kpkt), classify (the
        rest: classify, gamma, macro-atom queue binning, exact jumps, deactivations)."""
        ms = (C.c_double * 4)()
        nl = (C.c_int64 * 4)()
        self.lib.artis_gpu_last_kernel_times(ms, nl)
        return {k: (ms[i], nl[i]) for i, k in enumerate(("rpkt", "ma", "kpkt", "classify"))}

    KERNEL_CLASSES = ("rpkt", "ma", "kpkt", "classify", "binning", "exact", "finish")

    def last_kernel_class_times(self):
        """{class: (ms, launches)} for the last transport, finer than last_kernel_times: rpkt (k_rpkt), ma (k_ma),
        kpkt (k_kpkt), classify (k_classify + k_gamma), binning (the M-queue counting sort), exact (k_ma_exact),
        finish (k_ma_finish)."""
        n = len(self.KERNEL_CLASSES)
        ms = (C.c_double * n)()
        nl = (C.c_int64 * n)()
        self._check(self.lib.artis_gpu_last_kernel_class_times(ms, nl), "last_kernel_class_times")
        return {k: (ms[i], nl[i]) for i, k in enumerate(self.KERNEL_CLASSES)}

    # multi-GPU (RCCL): one communicator per engine, the packed estimator block all-reduced in HBM
    def comm_init(self, rank, nranks, uid):
        buf = C.create_string_buffer(bytes(uid), ffi.COMM_ID_BYTES)
        self._check(self.lib.artis_gpu_comm_init(int(rank), int(nranks), buf), "comm_init")

    def allreduce_estimators(self):
        self._check(self.lib.artis_gpu_estimators_allreduce(), "estimators_allreduce")

    def last_rounds(self):
        return int(self.lib.artis_gpu_last_rounds())

    def close(self):
        self.lib.artis_gpu_finalize()
