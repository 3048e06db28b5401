"""The C++ host mirror (artis_amd/csrc/host/update_packets_gpu.cc) driven by the sn3d-style timestep loop of
artis_amd/lib/artis_gpu_driver, without Python in the path.  The raw packet files it writes
(packets_0000_tsN.tmp, sn3d.cc:387-398) are checked against the CPU oracle run over the same timesteps."""
import os
import subprocess

import numpy as np
import pytest

import oracle_lib
import parity
from artis_amd import ffi

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DRIVER = os.path.join(REPO, "artis_amd", "lib", "artis_gpu_driver")
CFG = dict(ngrid_1d=10, nlevels_per_ion=60, n_ionising=20, max_lines=8000, ntstep=30)
NTS0, NSTEPS, NPKTS, SEED = 8, 2, 1500, 5


def _args(outdir):
    return [DRIVER, str(outdir), str(CFG["ngrid_1d"]), str(CFG["nlevels_per_ion"]), str(CFG["n_ionising"]),
            str(CFG["max_lines"]), str(CFG["ntstep"]), str(NTS0), str(NSTEPS), str(NPKTS), str(SEED)]


def test_driver_fails_loudly_without_gpu(tmp_path):
    """No silent CPU path: on a host without a usable GPU the C++ mirror aborts with the engine's message."""
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    r = subprocess.run(_args(tmp_path), capture_output=True, text=True, timeout=600)
    assert r.returncode != 0
    assert "artis_gpu_init failed" in r.stderr


@pytest.mark.gpu
def test_driver_matches_oracle(tmp_path):
    r = subprocess.run(_args(tmp_path), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr
    from artis_amd.model import Model

    m = Model(**CFG)
    m.set_timestep(NTS0)
    po = m.init_rpackets(NTS0, NPKTS, seed=SEED)
    for nts in range(NTS0, NTS0 + NSTEPS):
        m.set_timestep(nts)
        oracle_lib.update_packets(m, nts, po, nthreads=16)
        pg = np.fromfile(tmp_path / f"packets_0000_ts{nts}.tmp", dtype=ffi.PACKET_DTYPE)
        assert len(pg) == NPKTS
        parity.assert_packets_match(pg, po)
    # the final text packet list (packet.cc:152-196) reads back to the last raw records at %g precision
    from artis_amd import io

    back = np.zeros(NPKTS, dtype=ffi.PACKET_DTYPE)
    io.read_packets(str(tmp_path / "packets00_0000.out"), back)
    np.testing.assert_array_equal(back["number"], pg["number"])
    np.testing.assert_array_equal(back["type"], pg["type"])
    np.testing.assert_allclose(back["nu_rf"], pg["nu_rf"], rtol=1e-5)


@pytest.mark.gpu
def test_driver_rccl_reduced_path(tmp_path):
    """ARTIS_DRIVER_RCCL=1: the estimators pass through the RCCL all-reduce of the device block
    (update_packets_reduced, artis_gpu_estimators_allreduce) -- with one rank the sums are unchanged and the
    packets identical to the plain path."""
    a, b = tmp_path / "plain", tmp_path / "rccl"
    a.mkdir()
    b.mkdir()
    ra = subprocess.run(_args(a), capture_output=True, text=True, timeout=600)
    rb = subprocess.run(_args(b), capture_output=True, text=True, timeout=600,
                        env={**os.environ, "ARTIS_DRIVER_RCCL": "1"})
    assert ra.returncode == 0 and rb.returncode == 0, rb.stderr
    def summary(out):  # "nts N nesc N cmf_lum X gamma_dep X pellet_decays N Jsum X transport_ms X" per timestep
        rows = [ln.split() for ln in out.splitlines() if ln.startswith("nts ")]
        return np.array([[float(r[i]) for i in (1, 3, 5, 7, 9, 11)] for r in rows])

    sa, sb = summary(ra.stdout), summary(rb.stdout)
    assert sa.shape == (NSTEPS, 6)
    # float64 atomic sums: the order of accumulation differs between runs
    np.testing.assert_allclose(sb, sa, rtol=1e-12, atol=0)
    for nts in range(NTS0, NTS0 + NSTEPS):
        assert (a / f"packets_0000_ts{nts}.tmp").read_bytes() == (b / f"packets_0000_ts{nts}.tmp").read_bytes()


def _read_te_case(path, m):
    """te_case.bin of artis_gpu_driver (ARTIS_DRIVER_TE=1): length-prefixed arrays -- the previous state and the raw
    estimators, the parameters, then the prepared radiation field and the solution."""
    raw = open(path, "rb").read()
    pos = 0

    def arr(dt):
        nonlocal pos
        n = int(np.frombuffer(raw, np.int64, 1, pos)[0])
        pos += 8
        a = np.frombuffer(raw, dt, n, pos).copy()
        pos += n * np.dtype(dt).itemsize
        return a

    te = ffi.TeArrays(m, t_current=1.0)
    te.TR, te.W, te.TJ, te.Te, te.groundlevelpop = (arr(np.float32) for _ in range(5))
    nne_old, pf_old = arr(np.float32), arr(np.float32)
    te.mgi_list = arr(np.int32)
    te.thick = arr(np.int16)
    J, nuJ, ff, col, gam, bfh, te.vol_init = (arr(np.float64) for _ in range(7))
    te.elem_meanweight = arr(np.float32)
    t_current, tmin, deltat, tratmid = np.frombuffer(raw, np.float64, 4, pos)
    pos += 32
    te.params.t_current, te.params.tmin = float(t_current), float(tmin)
    prep = ffi.UgArrays(m, deltat=deltat, tratmid=tratmid)
    prep.J, prep.nuJ, prep.ffheating, prep.colheating, prep.gamma, prep.bfheating = J, nuJ, ff, col, gam, bfh
    prep.nne, prep.partfunct = nne_old, pf_old
    out = {}
    for k in ("TR", "W", "TJ", "Te", "groundlevelpop", "nne", "nnetot", "partfunct"):
        out[k] = arr(np.float32)
    for k in ("totalcooling", "cooling_contrib_ion", "rates"):
        out[k] = arr(np.float64)
    out["iters"] = arr(np.int32)
    return te, prep, out


@pytest.mark.gpu
def test_driver_update_grid_on_gpu_matches_oracle(tmp_path):
    """The C++ host loop with update_grid on the GPU -- the estimator preparation (PacketEngine::prepare_temperatures)
    from the run's own raw estimators, then the temperature / ionisation solution (solve_temperatures) -- replayed
    on the CPU oracle."""
    env = dict(os.environ, ARTIS_DRIVER_TE="1")
    r = subprocess.run(_args(tmp_path), capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr
    from artis_amd.model import Model

    m = Model(**CFG)
    m.set_timestep(NTS0 + NSTEPS - 1)
    te, prep, out = _read_te_case(os.path.join(tmp_path, "te_case.bin"), m)
    assert oracle_lib.prepare_temperatures(m, te, prep) == 0
    g = te.mgi_list
    assert len(g) > 0
    for a, k in ((prep.TR_out, "TR"), (prep.W_out, "W"), (prep.TJ_out, "TJ")):
        x, y = a[g].astype(np.float64), out[k][g].astype(np.float64)
        assert np.all(np.abs(x - y) <= 2.5e-7 * np.abs(x)), k
    te.TR, te.W, te.TJ = prep.TR_out.copy(), prep.W_out.copy(), prep.TJ_out.copy()
    te.ffheating, te.colheating = prep.ff_out.copy(), prep.col_out.copy()
    te.gamma, te.bfheating = prep.gamma_out.copy(), prep.bfheating_out.copy()
    assert oracle_lib.solve_temperatures(m, te) == 0
    same = (te.iters[g] == out["iters"][g]) & (np.abs(te.Te[g] - out["Te"][g]) <= 1e-9 * np.abs(te.Te[g]))
    assert same.mean() >= 0.99, same.mean()
    assert np.all(np.abs(te.Te[g] - out["Te"][g]) <= 2e-2 * np.abs(te.Te[g]))
    ok = g[same]
    for k in ("nne", "totalcooling"):
        a, b = getattr(te, k)[ok].astype(np.float64), out[k][ok].astype(np.float64)
        assert np.all(np.abs(a - b) <= 1e-6 * np.maximum(np.abs(a), np.abs(b)) + 1e-300), k
