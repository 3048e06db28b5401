"""Diagnostic: the uncached macro-atom walk on the nebular test model, step by step with timestamps."""
import faulthandler
import os
import sys
import time

_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [_R, os.path.join(_R, "tests")]
faulthandler.dump_traceback_later(60, repeat=True)
os.environ["ARTIS_GPU_NO_MACACHE"] = "1"
import oracle_lib  # noqa: E402
from artis_amd import Engine  # noqa: E402
from artis_amd.model import Model  # noqa: E402

NEB = dict(ngrid_1d=6, nlevels_per_ion=30, n_ionising=10, max_lines=2000, ntstep=20, nebular=1, nlte_level_max=12,
           tmin_days=100., tmax_days=300., T0=6000., ionpot_scale=0.5)
t0 = time.time()
m = Model(**NEB)
m.set_timestep(14)
pk = m.init_rpackets(14, 4000, seed=63)
print("model", time.time() - t0, flush=True)
po = pk.copy()
eo, wo = oracle_lib.update_packets(m, 14, po, nthreads=16)
print("oracle", time.time() - t0, wo[8], flush=True)
eng = Engine(m)
print("engine init", time.time() - t0, flush=True)
eng.upload_cellstate(14)
print("upload", time.time() - t0, flush=True)
pg = pk.copy()
eg = eng.update_packets(14, pg)
print("update", time.time() - t0, eng.last_work()[8], flush=True)
eng.close()
