"""The reference's run-input formats on the host (include/artis_io.h): input.txt, model.txt (1D / 3D) and
abundances.txt, read from the reference's own CI inputs (tests/golden/ref_inputs, copies of
tests/*_inputfiles) and from generated 3D files; plus the grid the model builder maps them onto
(map_1dmodeltogrid / map_3dmodeltogrid) and an oracle run on each reference model.  CPU only.
"""
import lzma
import os

import numpy as np
import pytest

import oracle_lib
from artis_amd import ffi, io
from artis_amd.model import Model

REF = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ref_inputs")
DAY = 86400.0


def _plain_model(tmp_path, name):
    d = os.path.join(REF, name)
    if os.path.exists(os.path.join(d, "model.txt.xz")):
        p = tmp_path / "model.txt"
        p.write_bytes(lzma.open(os.path.join(d, "model.txt.xz")).read())
        return str(p)
    return os.path.join(d, "model.txt")


def _data_rows(path):
    """Rows of a 1D model.txt by an independent parse: skip comment lines, npts, t_model, data."""
    lines = [ln for ln in open(path) if ln.strip() and not ln.lstrip().startswith("#")]
    npts = int(lines[0].split()[0])
    t_model = float(lines[1].split()[0])
    rows = [[float(x) for x in ln.split()] for ln in lines[2:2 + npts]]
    return npts, t_model, rows


def test_input_txt_classic():
    p = io.read_input_file(os.path.join(REF, "classicmode", "input-newrun.txt"))
    assert p.pre_zseed == 1281360349 and p.ntstep == 50 and (p.itstep, p.ftstep) == (0, 36)
    assert (p.tmin_days, p.tmax_days) == (3.0, 30.0) and p.model_type == 1
    assert p.rlc_mode == 4 and p.do_r_lc == 1 and p.do_rlc_est == 3  # input.cc:1976-1979
    assert p.gamma_grey == -1 and tuple(p.syn_dir) == (0.0, 0.0, 1.0) and p.opacity_case == 4
    assert p.num_lte_timesteps == 5 and p.cell_is_optically_thick == 8.0 and p.num_grey_timesteps == 999
    assert p.max_bf_continua == 1000000 and p.nprocs_exspec == 2 and p.do_emission_res == 1
    assert abs(p.kpktdiffusion_timescale - 0.001) < 1e-9 and p.n_kpktdiffusion_timesteps == 1000


def test_input_txt_kilonova_and_nebular():
    k = io.read_input_file(os.path.join(REF, "kilonova", "input-newrun.txt"))
    assert k.ntstep == 10 and (k.tmin_days, k.tmax_days) == (0.4, 10.0)
    assert k.num_lte_timesteps == 999 and k.cell_is_optically_thick == 0.0 and k.num_grey_timesteps == 5
    n = io.read_input_file(os.path.join(REF, "nebularonezone", "input-newrun.txt"))
    assert n.ntstep == 10 and (n.tmin_days, n.tmax_days) == (170.0, 230.0) and n.num_grey_timesteps == 4


@pytest.mark.parametrize("name,npts,t_model_days,custom", [("classicmode", 78, 0.976, False),
                                                           ("kilonova", 25, 0.05, True),
                                                           ("nebularonezone", 1, 0.000231481, False)])
def test_model_txt_1d(tmp_path, name, npts, t_model_days, custom):
    path = _plain_model(tmp_path, name)
    m = io.read_model(path, 1)
    n, t_model, rows = _data_rows(path)
    assert m["npts_model"] == npts == n and abs(m["t_model"] - t_model_days * DAY) < 1e-6 * DAY
    rows = np.array([r[:10] for r in rows])
    assert np.allclose(m["vout"], rows[:, 1] * 1e5, rtol=1e-12)
    assert np.allclose(m["rho_model"], 10 ** rows[:, 2], rtol=1e-12)
    assert np.allclose(m["ffegrp"], rows[:, 3]) and np.allclose(m["x_ni56"], rows[:, 4])
    assert m["vmax"] == m["vout"][-1]
    assert (m["n_custom_columns"] > 0) == custom


def test_abundances(tmp_path):
    path = os.path.join(REF, "classicmode", "abundances.txt")
    ab = io.read_abundances(path, 78, 1, [26, 27, 28, 8])
    raw = np.loadtxt(path)
    norm = raw[:, 1:].sum(axis=1)
    for j, z in enumerate([26, 27, 28, 8]):
        assert np.allclose(ab[:, j], raw[:, z] / norm, rtol=1e-6)
    # 3D models are not normalised (grid.cc:1052)
    ab3 = io.read_abundances(path, 78, 3, [26])
    assert np.allclose(ab3[:, 0], raw[:, 26].astype(np.float32))
    # wrong cell numbering fails
    bad = tmp_path / "ab.txt"
    bad.write_text("2 0.5 0.5\n")
    with pytest.raises(OSError):
        io.read_abundances(str(bad), 1, 1, [1])


def _write_3d(path, n, vmax, t_model_days, rho, zyx=False, abund7=False):
    xmax = vmax * t_model_days * DAY
    w = 2 * xmax / n
    with open(path, "w") as f:
        f.write(f"{n ** 3}\n{t_model_days}\n{vmax}\n")
        for i in range(n ** 3):
            c = (i % n, (i // n) % n, i // (n * n))
            pos = [-xmax + w * c[a] for a in range(3)]
            if zyx:
                pos = pos[::-1]
            f.write(f"{i + 1} {pos[0]:.6e} {pos[1]:.6e} {pos[2]:.6e} {rho[i]:.6e}\n")
            f.write("0.5 0.3 0.01 0.0 0.0" + (" 0.0 0.0\n" if abund7 else "\n"))


@pytest.mark.parametrize("zyx", [False, True])
def test_model_txt_3d(tmp_path, zyx):
    n = 6
    rng = np.random.default_rng(3)
    rho = rng.uniform(1e-14, 1e-12, n ** 3)
    rho[::7] = 0.0
    p = tmp_path / "model.txt"
    _write_3d(p, n, 1.0e9, 1.0, rho, zyx=zyx)
    m = io.read_model(str(p), 3)
    assert m["ncoord_model"] == (n, n, n) and m["posorder_zyx"] == int(zyx) and m["vmax"] == 1.0e9
    assert np.allclose(m["rho_model"], rho, rtol=1e-6)
    keep = rho > 0
    assert np.allclose(m["ffegrp"][keep], 0.5) and np.all(m["ffegrp"][~keep] == 0)
    # a cube-root mismatch or a missing abundance line fails loudly
    bad = tmp_path / "bad.txt"
    bad.write_text("10\n1.0\n1e9\n")
    with pytest.raises(OSError):
        io.read_model(str(bad), 3)


def test_model_from_files_3d_grid(tmp_path):
    """3D model.txt: the propagation grid is the model grid; empty cells map to npts_model (map_3dmodeltogrid)."""
    n = 6
    rng = np.random.default_rng(4)
    rho = rng.uniform(1e-14, 1e-12, n ** 3)
    rho[::5] = 0.0
    _write_3d(tmp_path / "model.txt", n, 1.0e9, 1.0, rho, abund7=True)
    with open(tmp_path / "abundances.txt", "w") as f:
        for i in range(n ** 3):
            f.write(f"{i + 1} " + " ".join(["0.0"] * 25) + " 0.6 0.1 0.3\n")
    inp = open(os.path.join(REF, "classicmode", "input-newrun.txt")).read().splitlines()
    inp[7] = "3                        # model_type"
    (tmp_path / "input.txt").write_text("\n".join(inp) + "\n")
    m = Model(files=(tmp_path / "input.txt", tmp_path / "model.txt", tmp_path / "abundances.txt"),
              ngrid_1d=99, nlevels_per_ion=20, n_ionising=8, max_lines=1000)
    assert m.cfg.ngrid_1d == n and m.npts_model == n ** 3
    m.set_timestep(5)
    pk = m.init_rpackets(5, 500, seed=1)
    assert np.all(rho[pk["where"]] > 0)  # packets start in non-empty cells
    est, _ = oracle_lib.update_packets(m, 5, pk, nthreads=4)
    assert est.struct.nesc == (pk["type"] == ffi.TYPE_ESCAPE).sum()


@pytest.mark.parametrize("name,ng,nts", [("classicmode", 30, 30), ("kilonova", 20, 5)])
def test_oracle_on_reference_models(name, ng, nts):
    """The oracle propagates the reference models: every surviving packet reaches t2, escaped-energy bookkeeping
    closes, macro-atom activations == deactivations (stats.h)."""
    d = os.path.join(REF, name)
    mf = os.path.join(d, "model.txt.xz" if name == "kilonova" else "model.txt")
    m = Model(files=(os.path.join(d, "input-newrun.txt"), mf, os.path.join(d, "abundances.txt")), ngrid_1d=ng,
              nlevels_per_ion=30, n_ionising=12, max_lines=3000, relativistic=int(name == "kilonova"))
    m.set_timestep(nts)
    pk = m.init_rpackets(nts, 800, seed=2)
    est, work = oracle_lib.update_packets(m, nts, pk, nthreads=4)
    esc = pk["type"] == ffi.TYPE_ESCAPE
    assert est.struct.nesc == esc.sum()
    assert np.isclose(est.struct.cmf_lum, pk["e_cmf"][esc].sum(), rtol=1e-12)
    assert np.all(pk["prop_time"][~esc] == pk["prop_time"][~esc].max())
    c = est.counters
    assert c[0] + c[1] + c[4] + c[5] == c[7] + c[8] + c[9] + c[10]
    assert work[2] > 0  # lines scanned
