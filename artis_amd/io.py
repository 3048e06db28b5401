"""ctypes mirror of include/artis_io.h: the reference's packet and virtual-packet file formats.

packets00_RRRR.out (packet.cc:152-196 / 211-290), packets_RRRR_tsN.tmp (sn3d.cc:387-398, packet.cc:198-209),
vspecpol (vpkt.cc:445-545) and vpkt_grid (vpkt.cc:629-665), implemented in C++ (artis_amd/csrc/host/artis_io.cc);
and the run inputs input.txt (input.cc:1874-2140), model.txt (grid.cc:1228-1370, 1459-1600) and abundances.txt
(grid.cc:1007-1073).
"""
import ctypes as C
import os

import numpy as np

from . import ffi

_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", "libartis_io.so")
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: run __graft_entry__.build()")
        L = C.CDLL(path)
        vp = C.c_void_p
        L.artis_write_packets.argtypes = [C.c_char_p, vp, C.c_int]
        L.artis_read_packets.argtypes = [C.c_char_p, vp, C.c_int]
        L.artis_write_temp_packetsfile.argtypes = [C.c_char_p, C.c_int, C.c_int, vp, C.c_int]
        L.artis_read_temp_packetsfile.argtypes = [C.c_char_p, C.c_int, C.c_int, vp, C.c_int]
        for fn in ("artis_write_vspecpol", "artis_read_vspecpol", "artis_read_vpkt_grid"):
            getattr(L, fn).argtypes = [C.c_char_p, C.POINTER(ffi.VpktParams), C.POINTER(ffi.VpktResult)]
        L.artis_write_vpkt_grid.argtypes = [C.c_char_p, C.POINTER(ffi.VpktParams), C.c_double,
                                            C.POINTER(ffi.VpktResult)]
        L.artis_read_input_file.argtypes = [C.c_char_p, C.POINTER(InputParams)]
        L.artis_read_model.argtypes = [C.c_char_p, C.c_int, C.POINTER(EjectaModel)]
        L.artis_free_model.argtypes = [C.POINTER(EjectaModel)]
        L.artis_free_model.restype = None
        L.artis_read_abundances.argtypes = [C.c_char_p, C.c_int, C.c_int, C.c_int, vp, vp]
        _LIB = L
    return _LIB


class InputParams(C.Structure):  # include/artis_io.h artis_input_params
    _fields_ = [
        ("pre_zseed", C.c_uint32), ("ntstep", C.c_int32), ("itstep", C.c_int32), ("ftstep", C.c_int32),
        ("tmin_days", C.c_double), ("tmax_days", C.c_double), ("nusyn_min_mev", C.c_double),
        ("nusyn_max_mev", C.c_double), ("nsyn_time", C.c_int32), ("syn_time_start_days", C.c_double),
        ("syn_time_dlog", C.c_double), ("model_type", C.c_int32), ("rlc_mode", C.c_int32), ("do_r_lc", C.c_int32),
        ("do_rlc_est", C.c_int32), ("n_out_it", C.c_int32), ("clight_factor", C.c_double),
        ("gamma_grey", C.c_double), ("syn_dir", C.c_double * 3), ("opacity_case", C.c_int32),
        ("rho_crit_para", C.c_double), ("debug_packet", C.c_int32), ("continued_from_saved", C.c_int32),
        ("rfcut_angstroms", C.c_double), ("num_lte_timesteps", C.c_int32), ("cell_is_optically_thick", C.c_double),
        ("num_grey_timesteps", C.c_int32), ("max_bf_continua", C.c_int32), ("nprocs_exspec", C.c_int32),
        ("do_emission_res", C.c_int32), ("kpktdiffusion_timescale", C.c_double),
        ("n_kpktdiffusion_timesteps", C.c_int32),
    ]


class EjectaModel(C.Structure):  # include/artis_io.h artis_ejecta_model
    _fields_ = [
        ("model_type", C.c_int32), ("npts_model", C.c_int32), ("ncoord_model", C.c_int32 * 3),
        ("t_model", C.c_double), ("vmax", C.c_double), ("vout", C.POINTER(C.c_double)),
        ("rho_model", C.POINTER(C.c_double)), ("ffegrp", C.POINTER(C.c_double)), ("x_ni56", C.POINTER(C.c_double)),
        ("x_co56", C.POINTER(C.c_double)), ("x_fe52", C.POINTER(C.c_double)), ("x_cr48", C.POINTER(C.c_double)),
        ("x_ni57", C.POINTER(C.c_double)), ("x_co57", C.POINTER(C.c_double)), ("pos_model", C.POINTER(C.c_float)),
        ("n_custom_columns", C.c_int32), ("posorder_zyx", C.c_int32),
    ]


def read_input_file(path):
    p = InputParams()
    _ok(lib().artis_read_input_file(os.fspath(path).encode(), C.byref(p)), "artis_read_input_file")
    return p


def read_model(path, model_type):
    """model.txt -> dict of numpy arrays (copies) + scalars."""
    m = EjectaModel()
    _ok(lib().artis_read_model(os.fspath(path).encode(), int(model_type), C.byref(m)), "artis_read_model")
    try:
        n = m.npts_model
        out = {"model_type": m.model_type, "npts_model": n, "ncoord_model": tuple(m.ncoord_model),
               "t_model": m.t_model, "vmax": m.vmax, "n_custom_columns": m.n_custom_columns,
               "posorder_zyx": m.posorder_zyx}
        for f in ("rho_model", "ffegrp", "x_ni56", "x_co56", "x_fe52", "x_cr48", "x_ni57", "x_co57"):
            out[f] = np.ctypeslib.as_array(getattr(m, f), shape=(n,)).copy()
        out["vout"] = np.ctypeslib.as_array(m.vout, shape=(n,)).copy() if m.vout else None
        out["pos_model"] = np.ctypeslib.as_array(m.pos_model, shape=(n, 3)).copy() if m.pos_model else None
    finally:
        lib().artis_free_model(C.byref(m))
    return out


def read_abundances(path, npts_model, model_type, anumbers):
    an = np.ascontiguousarray(np.asarray(anumbers, dtype=np.int32))
    out = np.zeros((npts_model, len(an)), dtype=np.float32)
    _ok(lib().artis_read_abundances(os.fspath(path).encode(), int(npts_model), int(model_type), len(an),
                                    an.ctypes.data, out.ctypes.data), "artis_read_abundances")
    return out


def _ok(rc, what):
    if rc != 0:
        raise OSError(f"{what} -> {rc}")


def write_packets(path, pk):
    _ok(lib().artis_write_packets(path.encode(), pk.ctypes.data, len(pk)), "artis_write_packets")


def read_packets(path, pk):
    _ok(lib().artis_read_packets(path.encode(), pk.ctypes.data, len(pk)), "artis_read_packets")


def write_temp_packetsfile(directory, timestep, rank, pk):
    _ok(lib().artis_write_temp_packetsfile(directory.encode(), timestep, rank, pk.ctypes.data, len(pk)),
        "artis_write_temp_packetsfile")


def read_temp_packetsfile(directory, timestep, rank, pk):
    _ok(lib().artis_read_temp_packetsfile(directory.encode(), timestep, rank, pk.ctypes.data, len(pk)),
        "artis_read_temp_packetsfile")


def write_vspecpol(path, cfg, arrays):
    _ok(lib().artis_write_vspecpol(path.encode(), C.byref(cfg.struct), C.byref(arrays.struct)), "artis_write_vspecpol")


def read_vspecpol(path, cfg, arrays):
    _ok(lib().artis_read_vspecpol(path.encode(), C.byref(cfg.struct), C.byref(arrays.struct)), "artis_read_vspecpol")


def write_vpkt_grid(path, cfg, vmax, arrays):
    _ok(lib().artis_write_vpkt_grid(path.encode(), C.byref(cfg.struct), float(vmax), C.byref(arrays.struct)),
        "artis_write_vpkt_grid")


def read_vpkt_grid(path, cfg, arrays):
    _ok(lib().artis_read_vpkt_grid(path.encode(), C.byref(cfg.struct), C.byref(arrays.struct)), "artis_read_vpkt_grid")
