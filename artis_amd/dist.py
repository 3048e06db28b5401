"""Multi-GPU estimator reduction: the reference's mpi_reduce_estimators (sn3d.cc:582, radfield.cc:1502-1564,
sn3d.cc:316-377) as ONE all-reduce of one packed float64 block per timestep.

Each rank propagates its own full-energy packet ensemble (packet.cc:106-149; rank-specific RNG key), so the
only exchange is a SUM of the estimator accumulators.  The block layout is the engine's device layout
(engine.hip artis_gpu_estimator_block_to_device):
  [J | nuJ | ffheating | colheating (npts_model each) | gammaestimator | bfheatingestimator (npts*E*I each)
   | time_step scalars (8) | ecounter | acounter (nlines each) | counters (34) | nesc]
Counts travel as float64 (exact below 2**53).  On GPUs the block is reduced in HBM over RCCL/xGMI
(torch.distributed "nccl"); the same layout is reduced on host arrays with "gloo" in the CPU tests.
"""
import numpy as np

from . import ffi


def block_len(npts_model, nelements, maxnions, nlines):
    return 4 * npts_model + 2 * npts_model * nelements * maxnions + 8 + 2 * nlines + ffi.ARTIS_COUNTER_COUNT + 1


def pack_estimators(est):
    """EstimatorArrays -> float64 block (host mirror of the device layout)."""
    s = est.struct
    scal = np.array([s.cmf_lum, s.gamma_dep, s.positron_dep, s.electron_dep, s.electron_emission, s.alpha_dep,
                     s.alpha_emission, s.gamma_emission])
    return np.concatenate([est.J, est.nuJ, est.ffheating, est.colheating, est.gamma, est.bfheating, scal,
                           est.ecounter.astype(np.float64), est.acounter.astype(np.float64),
                           est.counters.astype(np.float64), np.array([float(s.nesc)])])


def unpack_estimators(block, est):
    """float64 block -> EstimatorArrays (overwrites)."""
    n = len(est.J)
    ni = len(est.gamma)
    nl = len(est.ecounter)
    o = 0
    for arr in (est.J, est.nuJ, est.ffheating, est.colheating):
        arr[:] = block[o:o + n]
        o += n
    for arr in (est.gamma, est.bfheating):
        arr[:] = block[o:o + ni]
        o += ni
    s = est.struct
    (s.cmf_lum, s.gamma_dep, s.positron_dep, s.electron_dep, s.electron_emission, s.alpha_dep, s.alpha_emission,
     s.gamma_emission) = [float(x) for x in block[o:o + 8]]
    o += 8
    est.ecounter[:] = np.rint(block[o:o + nl]).astype(np.int32)
    o += nl
    est.acounter[:] = np.rint(block[o:o + nl]).astype(np.int32)
    o += nl
    for k in range(ffi.ARTIS_COUNTER_COUNT):
        s.counters[k] = int(round(block[o + k]))
    o += ffi.ARTIS_COUNTER_COUNT
    s.nesc = int(round(block[o]))
    return est


def allreduce_engine_estimators(engine, torch_buffer, dist_module):
    """Sum the device estimator blocks of all ranks in place (RCCL over xGMI when backend is nccl)."""
    engine.estimator_block_to_device(torch_buffer.data_ptr())
    dist_module.all_reduce(torch_buffer)
    engine.estimator_block_from_device(torch_buffer.data_ptr())
