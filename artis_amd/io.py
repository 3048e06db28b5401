"""ctypes mirror of include/artis_io.h: the reference's packet and virtual-packet file formats.

packets00_RRRR.out (packet.cc:152-196 / 211-290), packets_RRRR_tsN.tmp (sn3d.cc:387-398, packet.cc:198-209),
vspecpol (vpkt.cc:445-545) and vpkt_grid (vpkt.cc:629-665), implemented in C++ (artis_amd/csrc/host/artis_io.cc).
"""
import ctypes as C
import os

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
        _LIB = L
    return _LIB


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
