"""Multi-GPU estimator reduction: the reference's mpi_reduce_estimators (sn3d.cc:582, radfield.cc:1502-1564,
sn3d.cc:316-377) as ONE all-reduce of one packed float64 block per timestep.

Each rank propagates its own full-energy packet ensemble (packet.cc:106-149; rank-specific RNG key), so the
only exchange is a SUM of the estimator accumulators.  The block layout is defined once, by the engine library
(include/artis_gpu.h: artis_gpu_estimator_block_to_device on the device, artis_estimator_block_pack / _unpack on
the host), and used here unchanged:
  [J | nuJ | ffheating | colheating | rpkt_emiss | gammaestimator | bfheatingestimator | 10 time_step scalars
   | bfrate_raw | radfield bins J, nuJ, contribcount (nebular options) | ecounter | acounter | counters (34) | nesc]
After the sum the eight time_step scalars are divided by the rank count, as mpi_reduce_estimators does
(sn3d.cc:370-377); everything else stays a sum (update_grid normalises by nprocs, update_grid.cc:1041).
On GPUs the block is all-reduced in HBM by the engine's own RCCL communicator over xGMI
(artis_gpu_comm_init / artis_gpu_estimators_allreduce; Engine.comm_init / Engine.allreduce_estimators);
host arrays are packed with the same layout and reduced with gloo in the CPU tests.
"""
import ctypes as C

import numpy as np

from . import gpu_lib


def block_len(npts_model, nelements, maxnions, nlines, nbf_est=0, nbins_est=0):
    return int(gpu_lib().artis_estimator_block_len(npts_model, nelements, maxnions, nlines, nbf_est, nbins_est))


def _dims(est):
    return est.npts_model, est.nelements, est.maxnions, len(est.ecounter), est.nbfcontinua, est.radfield_nbins


def pack_estimators(est):
    """ffi.EstimatorArrays -> float64 block in the device layout (artis_estimator_block_pack)."""
    dims = _dims(est)
    block = np.zeros(block_len(*dims))
    rc = gpu_lib().artis_estimator_block_pack(C.byref(est.struct), *dims, block.ctypes.data)
    if rc != 0:
        raise RuntimeError(f"artis_estimator_block_pack -> {rc}")
    return block


def unpack_estimators(block, est):
    """float64 block -> ffi.EstimatorArrays (overwrites; artis_estimator_block_unpack)."""
    dims = _dims(est)
    block = np.ascontiguousarray(block, dtype=np.float64)
    if len(block) != block_len(*dims):
        raise ValueError("estimator block length does not match the estimator arrays")
    rc = gpu_lib().artis_estimator_block_unpack(block.ctypes.data, *dims, C.byref(est.struct))
    if rc != 0:
        raise RuntimeError(f"artis_estimator_block_unpack -> {rc}")
    return est


def average_timestep_scalars(block, est, nranks):
    """After the SUM over nranks: the eight time_step scalars divided by nranks, as mpi_reduce_estimators does
    (sn3d.cc:370-377; artis_estimator_block_average_scalars).  The device all-reduce does the same in HBM."""
    block = np.ascontiguousarray(block, dtype=np.float64)
    rc = gpu_lib().artis_estimator_block_average_scalars(block.ctypes.data, est.npts_model, est.nelements,
                                                          est.maxnions, int(nranks))
    if rc != 0:
        raise RuntimeError(f"artis_estimator_block_average_scalars -> {rc}")
    return block


def join(engine, rank, world, dist_module):
    """Every rank joins the engine's RCCL communicator; rank 0's id travels over dist_module (any backend)."""
    from . import comm_unique_id

    obj = [comm_unique_id() if rank == 0 else None]
    dist_module.broadcast_object_list(obj, src=0)
    engine.comm_init(rank, world, obj[0])


def allreduce_engine_estimators(engine):
    """Sum the device estimator blocks of all ranks in place (RCCL over xGMI, engine stream); the eight time_step
    scalars are then divided by the rank count (sn3d.cc:370-377)."""
    engine.allreduce_estimators()
