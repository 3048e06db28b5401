"""The reference's file formats written / read by the host library (include/artis_io.h).  CPU only.

Each writer is checked line for line against an independent Python rendering of the reference's printf
format (packet.cc:152-196, vpkt.cc:445-483, 629-646), and each reader against its writer (round trip at the
precision of the text format; bit-exact for the raw .tmp records).
"""
import os

import numpy as np

import oracle_lib
from artis_amd import ffi, io
from artis_amd.model import Model


def _g(x):
    return "%g" % x


def _packet_line(p):
    """packet.cc:155-194 rendered in Python (%lg == %g for a double)."""
    f = []
    f += ["%d" % p["number"], "%d" % p["where"], "%d" % p["type"]]
    f += [_g(v) for v in p["pos"]] + [_g(v) for v in p["dir"]]
    f += ["%d" % p["last_cross"], _g(p["tdecay"]), _g(p["e_cmf"]), _g(p["e_rf"]), _g(p["nu_cmf"]), _g(p["nu_rf"])]
    f += ["%d" % p[k] for k in ("escape_type", "escape_time", "scat_count", "next_trans", "interactions",
                                 "last_event", "emissiontype", "trueemissiontype")]
    f += [_g(v) for v in p["em_pos"]]
    f += ["%d" % p["absorptiontype"], _g(p["absorptionfreq"]), "%d" % p["nscatterings"], "%d" % p["em_time"]]
    f += [_g(v) for v in p["absorptiondir"]] + [_g(v) for v in p["stokes"]] + [_g(v) for v in p["pol_dir"]]
    f += ["%d" % p["originated_from_particlenotgamma"], _g(float(p["trueemissionvelocity"])),
          "%d" % p["trueem_time"], "%d" % p["pellet_nucindex"]]
    return " ".join(f) + " "


def _evolved_packets(n=200):
    m = Model(ngrid_1d=6, nlevels_per_ion=20, n_ionising=8, max_lines=1500, ntstep=20)
    m.set_timestep(14)
    pk = m.init_rpackets(14, n, seed=51)
    oracle_lib.update_packets(m, 14, pk, nthreads=4)
    return pk


def test_packets_text_file_format_and_round_trip(tmp_path):
    pk = _evolved_packets()
    path = str(tmp_path / "packets00_0000.out")
    io.write_packets(path, pk)
    lines = open(path).read().split("\n")
    assert lines[0].startswith("#number where type_id posx")
    for i in (0, 7, len(pk) - 1):
        assert lines[1 + i] == _packet_line(pk[i])
    back = np.zeros_like(pk)
    io.read_packets(path, back)
    for name in ("number", "where", "type", "last_cross", "escape_type", "next_trans", "interactions", "last_event",
                 "emissiontype", "trueemissiontype", "absorptiontype", "nscatterings", "em_time", "trueem_time",
                 "pellet_nucindex", "escape_time", "scat_count"):
        np.testing.assert_array_equal(back[name], pk[name], err_msg=name)
    for name in ("pos", "dir", "e_cmf", "e_rf", "nu_cmf", "nu_rf", "stokes", "absorptionfreq"):
        ref = np.vectorize(lambda x: float(_g(x)))(pk[name])
        np.testing.assert_array_equal(back[name], ref, err_msg=name)
    short = np.zeros(len(pk) + 1, dtype=ffi.PACKET_DTYPE)
    try:
        io.read_packets(path, short)
        raise AssertionError("a short packets file must be rejected (packet.cc:283-288)")
    except OSError:
        pass


def test_temp_packets_file_is_raw_records(tmp_path):
    pk = _evolved_packets(64)
    io.write_temp_packetsfile(str(tmp_path), 14, 3, pk)
    path = tmp_path / "packets_0003_ts14.tmp"
    assert os.path.getsize(path) == 304 * len(pk)
    assert path.read_bytes() == pk.tobytes()
    back = np.zeros_like(pk)
    io.read_temp_packetsfile(str(tmp_path), 14, 3, back)
    assert back.tobytes() == pk.tobytes()


def test_vspecpol_and_vpkt_grid_files(tmp_path):
    vc = ffi.VpktConfig(nz_obs=(0.3, -0.5), phi_obs_deg=(0.0, 90.0), exclude=(0.0, -1.0), vmtbins=5, vmnubins=7,
                        vgrid=True, ny_vgrid=4, nz_vgrid=3, grid_ranges_angstrom=((3500.0, 6000.0), (6000.0, 9000.0)))
    a = ffi.VpktArrays(vc)
    rng = np.random.default_rng(5)
    a.vstokes[...] = rng.lognormal(size=a.vstokes.shape) * 1e-3
    a.vgrid[...] = rng.normal(size=a.vgrid.shape) * 1e40
    path = str(tmp_path / "vspecpol_0-0.out")
    io.write_vspecpol(path, vc, a)
    rows = [r.split() for r in open(path).read().strip().split("\n")]
    ncomb = 4
    assert len(rows) == ncomb * (1 + 7)
    lt, dt, lf, df = vc.bins()
    header = ["0"] + [_g((float(lt[t]) + float(dt[t]) / 2.0) / ffi.DAY) for t in range(5)] * 3
    assert rows[0] == header
    # row of ind_comb 1, frequency bin 2: nu centre, then I, Q, U over the 5 time bins
    r = rows[8 + 1 + 2]
    assert r[0] == _g(float(lf[2]) + float(df[2]) / 2.0)
    assert r[1:] == [_g(a.vstokes[l, t, 1, 2]) for l in range(3) for t in range(5)]
    b = ffi.VpktArrays(vc)
    io.read_vspecpol(path, vc, b)
    np.testing.assert_array_equal(b.vstokes, np.vectorize(lambda x: float(_g(x)))(a.vstokes))
    gpath = str(tmp_path / "vpkt_grid_0-0.out")
    vmax = 1e9
    io.write_vpkt_grid(gpath, vc, vmax, a)
    grows = [r.split() for r in open(gpath).read().strip().split("\n")]
    assert len(grows) == 2 * 2 * 4 * 3
    # obs 1, range 0, n 2, m 1 (vpkt.cc:630-643 loop order: obs, range, n, m)
    k = ((1 * 2 + 0) * 4 + 2) * 3 + 1
    assert grows[k] == [_g(vmax - 2.5 * 2 * vmax / 4), _g(vmax - 1.5 * 2 * vmax / 3),
                        _g(a.vgrid[0, 2, 1, 0, 1]), _g(a.vgrid[1, 2, 1, 0, 1]), _g(a.vgrid[2, 2, 1, 0, 1])]
    c = ffi.VpktArrays(vc)
    io.read_vpkt_grid(gpath, vc, c)
    np.testing.assert_array_equal(c.vgrid, np.vectorize(lambda x: float(_g(x)))(a.vgrid))
