"""The drop-in boundary: packet record layout, exported symbols, struct mirrors.  CPU only."""
import ctypes as C
import os
import re
import subprocess
import tempfile

import numpy as np

from artis_amd import ABI_SYMBOLS, GPU_SO, ffi

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "artis_gpu.h")

# reference offsets of struct packet (packet.h:28-73, probed sizeof 304)
REF_OFFSETS = {"where": 0, "type": 4, "pos": 24, "dir": 48, "e_cmf": 72, "e_rf": 80, "nu_cmf": 88, "nu_rf": 96,
               "next_trans": 104, "prop_time": 144, "stokes": 200, "tdecay": 248, "mastate": 288}


def test_packet_dtype_matches_reference_offsets():
    assert ffi.PACKET_DTYPE.itemsize == 304
    for name, off in REF_OFFSETS.items():
        assert ffi.PACKET_DTYPE.fields[name][1] == off, name


def _c_layout():
    """Compile a probe against include/artis_gpu.h and return sizeof/offsetof values."""
    src = r"""
#include <stdio.h>
#include <stddef.h>
#include "artis_gpu.h"
#define O(f) printf(#f " %zu\n", offsetof(artis_packet, f));
int main(void) {
  printf("sizeof %zu\n", sizeof(artis_packet));
  O(where) O(type) O(last_cross) O(interactions) O(nscatterings) O(last_event) O(pos) O(dir) O(e_cmf) O(e_rf)
  O(nu_cmf) O(nu_rf) O(next_trans) O(emissiontype) O(em_pos) O(em_time) O(prop_time) O(absorptiontype)
  O(trueemissiontype) O(trueem_time) O(absorptionfreq) O(absorptiondir) O(stokes) O(pol_dir) O(tdecay)
  O(escape_type) O(escape_time) O(scat_count) O(number) O(originated_from_particlenotgamma) O(pellet_decaytype)
  O(pellet_nucindex) O(trueemissionvelocity) O(mastate) O(_pad0) O(_pad1) O(_pad2)
  printf("estimators %zu\n", sizeof(artis_estimators));
  printf("run_params %zu\n", sizeof(artis_run_params));
  printf("cell_state %zu\n", sizeof(artis_cell_state));
  printf("gamma_spectra %zu\n", sizeof(artis_gamma_spectra));
  printf("vpkt_params %zu\n", sizeof(artis_vpkt_params));
  printf("vpkt_result %zu\n", sizeof(artis_vpkt_result));
  printf("vpkt_tau_max %zu\n", offsetof(artis_vpkt_params, tau_max_vpkt));
  printf("vpkt_spawn_capacity %zu\n", offsetof(artis_vpkt_params, spawn_capacity));
  printf("te_params %zu\n", sizeof(artis_te_params));
  printf("te_cells %zu\n", sizeof(artis_te_cells));
  printf("te_cells_te_iterations %zu\n", offsetof(artis_te_cells, te_iterations));
  printf("ug_prepare %zu\n", sizeof(artis_ug_prepare));
  printf("ug_prepare_renorm %zu\n", offsetof(artis_ug_prepare, corrphotoionrenorm_out));
  return 0;
}
"""
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "probe.c")
        exe = os.path.join(d, "probe")
        open(c, "w").write(src)
        subprocess.run(["gcc", "-std=c99", "-I" + os.path.join(REPO, "include"), c, "-o", exe], check=True)
        out = subprocess.run([exe], check=True, capture_output=True, text=True).stdout
    return {ln.split()[0]: int(ln.split()[1]) for ln in out.strip().splitlines()}


def test_c_header_layout_matches_numpy_and_ctypes():
    lay = _c_layout()
    assert lay["sizeof"] == 304
    for name in ffi.PACKET_DTYPE.names:
        assert lay[name] == ffi.PACKET_DTYPE.fields[name][1], name
    assert lay["estimators"] == C.sizeof(ffi.Estimators)
    assert lay["run_params"] == C.sizeof(ffi.RunParams)
    assert lay["gamma_spectra"] == C.sizeof(ffi.GammaSpectra)
    assert lay["vpkt_params"] == C.sizeof(ffi.VpktParams)
    assert lay["vpkt_result"] == C.sizeof(ffi.VpktResult)
    assert lay["vpkt_tau_max"] == ffi.VpktParams.tau_max_vpkt.offset
    assert lay["vpkt_spawn_capacity"] == ffi.VpktParams.spawn_capacity.offset
    assert lay["te_params"] == C.sizeof(ffi.TeParams)
    assert lay["te_cells"] == C.sizeof(ffi.TeCells)
    assert lay["te_cells_te_iterations"] == ffi.TeCells.te_iterations.offset
    assert lay["ug_prepare"] == C.sizeof(ffi.UgPrepare)
    assert lay["ug_prepare_renorm"] == ffi.UgPrepare.corrphotoionrenorm_out.offset
    assert lay["cell_state"] == 24 * 8  # 15 array pointers + ffegrp + 8 nebular (ABI 6)


def test_header_declares_exactly_the_abi_symbols():
    text = open(HEADER).read()
    declared = set(re.findall(r"\b(artis_(?:gpu|estimator)_\w+)\s*\(", text))
    assert declared == set(ABI_SYMBOLS)


def test_library_exports_every_declared_symbol():
    assert os.path.exists(GPU_SO), "libartis_gpu.so not built"
    out = subprocess.run(["nm", "-D", "--defined-only", GPU_SO], check=True, capture_output=True, text=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if ln.strip()}
    missing = [s for s in ABI_SYMBOLS if s not in exported]
    assert not missing, missing


def test_library_loads_without_gpu_and_reports_version():
    lib = C.CDLL(GPU_SO)
    assert lib.artis_gpu_abi_version() == 11
    lib.artis_gpu_last_error.restype = C.c_char_p
    assert lib.artis_gpu_last_error() is not None


def test_engine_refuses_uninitialised_calls():
    lib = C.CDLL(GPU_SO)
    lib.artis_gpu_update_packets_resident.argtypes = [C.c_int, C.c_int]
    assert lib.artis_gpu_update_packets_resident(0, 0) == -1  # ARTIS_ERR_NOT_INITIALISED


def test_raw_tmp_packet_file_roundtrip(tmp_path, small_model):
    """packets_RRRR_tsN.tmp is a raw fwrite of the 304-byte records (sn3d.cc:387-398, packet.cc:198-209)."""
    pk = small_model.init_rpackets(3, 37, seed=11)
    f = tmp_path / "packets_0000_ts3.tmp"
    pk.tofile(f)
    assert os.path.getsize(f) == 37 * 304
    back = np.fromfile(f, dtype=ffi.PACKET_DTYPE)
    assert back.tobytes() == pk.tobytes()


def test_init_refuses_unsupported_run_params():
    """artis_gpu_init returns ARTIS_ERR_UNSUPPORTED (before touching the GPU) for option values the engine does not
    propagate, instead of accepting and ignoring them: do_rlc_est outside 0..3 (input.cc:1976-1982), opacity_case
    outside 0..5 (grid.cc:627-677), a switch that is not 0/1."""
    from artis_amd import gpu_lib
    from artis_amd.model import Model

    m = Model(ngrid_1d=4, nlevels_per_ion=10, n_ionising=4, max_lines=200, ntstep=10)
    L = gpu_lib()
    for field, val in (("do_rlc_est", 4), ("do_rlc_est", -1), ("opacity_case", 6), ("pol_dipole", 2),
                       ("nlte_pops_on", 7), ("comp_est", -1), ("max_path_step", 0.0)):
        p = ffi.RunParams.from_buffer_copy(m.params)
        setattr(p, field, val)
        rc = L.artis_gpu_init(0, m.atomic, m.geometry, C.byref(p))
        assert rc == -6, (field, rc)  # ARTIS_ERR_UNSUPPORTED (include/artis_gpu.h)
        assert L.artis_gpu_last_error().decode(), field
