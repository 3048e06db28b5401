"""Two engines' device estimator blocks through a collective.  Needs an MI355X.

The multi-GPU path exchanges exactly one thing per timestep: the SUM of the ranks' estimator accumulators
(mpi_reduce_estimators, sn3d.cc:582 / radfield.cc:1502-1564), as one packed float64 block in HBM.  On the one-GPU
box two rank processes share the card: each runs its own engine (rank-specific RNG key, its own packets), writes its
device block (artis_gpu_estimator_block_to_device), the blocks are summed over gloo (RCCL needs one device per
rank), the eight time_step scalars averaged (sn3d.cc:370-377), and each engine reads the sum back
(artis_gpu_estimator_block_from_device).  The estimators each rank then downloads must be the oracle's two-rank sum.
"""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

CFG = dict(ngrid_1d=8, nlevels_per_ion=40, n_ionising=15, max_lines=3000, ntstep=30)
NTS = 5
NPKTS = 3000


def _worker(rank, world, port, outdir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist

    from artis_amd import Engine, ffi
    from artis_amd import dist as adist
    from artis_amd.model import Model

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        m = Model(**CFG)
        m.set_timestep(NTS)
        pk = m.init_rpackets(NTS, NPKTS, seed=1000 + rank)
        p = ffi.RunParams.from_buffer_copy(m.params)
        p.rank = rank
        eng = Engine(m, params=p)
        try:
            eng.upload_cellstate(NTS)
            eng.upload(pk)
            eng.zero_estimators()
            eng.step_resident(NTS, my_rank=rank)
            blk = torch.zeros(eng.estimator_block_doubles(), dtype=torch.float64, device="cuda")
            eng.estimator_block_to_device(blk.data_ptr())
            h = blk.cpu()
            dist.all_reduce(h)
            h = torch.from_numpy(adist.average_timestep_scalars(h.numpy(), m.new_estimators(), world))
            blk.copy_(h.to("cuda"))
            torch.cuda.synchronize()
            eng.estimator_block_from_device(blk.data_ptr())
            est = eng.download_estimators()
            np.savez(os.path.join(outdir, f"rank{rank}.npz"), J=est.J, nuJ=est.nuJ, ff=est.ffheating,
                     counters=est.counters, nesc=est.struct.nesc, cmf_lum=est.struct.cmf_lum)
            pg = pk.copy()
            eng.download(pg)
            np.save(os.path.join(outdir, f"pk{rank}.npy"), pg.view(np.uint8))
        finally:
            eng.close()
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_two_engines_device_blocks_allreduce(tmp_path):
    import torch.multiprocessing as mp

    import oracle_lib
    import parity
    from artis_amd import ffi
    from artis_amd.model import Model

    mp.start_processes(_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True, start_method="spawn")
    r0, r1 = np.load(tmp_path / "rank0.npz"), np.load(tmp_path / "rank1.npz")
    for k in ("J", "nuJ", "ff", "counters"):
        assert np.array_equal(r0[k], r1[k]), k  # both ranks hold the reduced block
    m = Model(**CFG)
    m.set_timestep(NTS)
    eo = m.new_estimators()
    for rank in (0, 1):
        po = m.init_rpackets(NTS, NPKTS, seed=1000 + rank)
        p = ffi.RunParams.from_buffer_copy(m.params)
        p.rank = rank
        oracle_lib.update_packets(m, NTS, po, est=eo, params=p, nthreads=16)  # (adds into eo)
        pg = np.load(tmp_path / f"pk{rank}.npy").view(po.dtype)
        parity.assert_packets_match(pg, po)  # each rank's own histories
    for k, ref in (("J", eo.J), ("nuJ", eo.nuJ), ("ff", eo.ffheating)):
        scale = max(np.abs(ref).max(), 1e-300)
        assert np.abs(r0[k] - ref).max() <= parity.ESTIMATOR_RTOL * scale, k
    assert parity.counters_equal(r0["counters"], eo.counters)
    assert int(r0["nesc"]) == eo.struct.nesc > 0
    # the eight time_step scalars are averaged over the ranks (sn3d.cc:370-377)
    assert abs(float(r0["cmf_lum"]) - eo.struct.cmf_lum / 2) <= 1e-9 * eo.struct.cmf_lum
