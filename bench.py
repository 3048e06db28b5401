"""bench.py -- packet-timesteps per second of the MI355X update_packets engine on the synthetic 50^3 grid.

python bench.py --gpus N --steps K --warmup W

N>1: one process per GPU.  Under torch.distributed.run (RANK / WORLD_SIZE set) this process is one rank; a bare
`python bench.py --gpus N` starts the N rank processes itself (before anything touches torch or the GPU), waits for
them and exits with their status -- rank 0 prints the JSON line.  --dry-launch does the same rank bring-up without a
GPU (gloo only) and prints the ranks that joined, for the CPU test of the launcher.

One step = one update_packets(nts) of this rank's P resident packets, all in HBM before timing starts:
  packets reset to the same initial ensemble (device-to-device copy), estimators zeroed, the per-timestep cell
  precompute (artis_gpu_upload_cellstate: cell-state H2D + per-cell table kernels), the transport kernel, and
  for N>1 the RCCL all-reduce of the packed estimator block (radfield J/nuJ, heating/photoionisation
  estimators, line statistics, event counters) -- the reference's mpi_reduce_estimators (sn3d.cc:582).
Packets are sharded: every rank propagates its own full-energy ensemble (rank-specific seed and RNG key), so
per-GPU work is fixed as N grows ("weak").  value = N * P * K / max-over-ranks wall time.

roofline: the dominant kernel class of the step (k_ma, k_rpkt, or k_vpkt with --vpkt): its algorithmic bytes
per launch / its average launch time, measured with HIP events around every launch on the engine stream,
against 8.0 TB/s.  Bytes: SURVEY.md §8(d)'s per-unit figures over the engine's own event counters, split by
the kernel that does the work, except that a macro-atom transition probe of the cached walk (a binary-search
step over running sums) is charged the 8 bytes it reads, not §8(d)'s 40-byte transition record
("achieved"); the §8(d) figure is reported beside it ("achieved_survey_model").  traffic: measured HBM bytes
per launch of that kernel (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, profiles/pmc_*.json), used only when the
summary was made from the same engine sources (engine_src_sha) and configuration.
cpu_baseline: the CPU oracle (oracle/liboracle.so, OpenMP) on a bounded sample of the same workload, rank 0
at N=1 only, on the CPU share this process may use (affinity and cgroup quota; host CPU model recorded).
N>1: ranks join the engine's RCCL communicator (rank 0's id broadcast over a gloo process group that also
provides the barriers and the max-over-ranks time); the estimator block is all-reduced in HBM by the engine
(artis_gpu_estimators_allreduce).
"""
import argparse
import glob
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "MC packets/sec/timestep on 50^3 grid; emergent-spectrum L1 vs CPU ref"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table: 8.0 TB/s spec


def byte_model(work, nions_total, probe_bytes=8.0):
    """Algorithmic bytes per kernel class from the work counters (include/artis_constants.h enum artis_work),
    SURVEY.md §8(d) per-unit figures: the r-packet kernel reads/writes the record, steps, scans lines, evaluates
    kappa and estimators; the macro-atom kernel reads a 72-byte rate record per jump and probe_bytes per
    transition probe (8: the running sum a binary-search step of the cached walk reads; §8(d) charges 40);
    the k-packet kernel scans cooling terms."""
    w = [float(x) for x in work]
    rpkt = (608.0 * w[0] + 168.0 * w[1] + 64.0 * w[2] + 88.0 * w[5] + 8.0 * nions_total * w[4] + 48.0 * w[6]
            + 32.0 * w[7])
    ma = 72.0 * w[8] + probe_bytes * w[9]
    kpkt = 16.0 * w[11]
    # macro-atom activations (bound-bound + continuum absorptions): each is binned into the cell-sorted queue
    # (queue slot, key, the packet's cell / level / number words, side state, the 32-byte ticket: 128 B) and
    # deactivated by k_ma_finish (the 304-byte packet record read and written: 608 B + side state 32 B)
    acts = w[14] + w[15]
    return {"rpkt": rpkt, "ma": ma, "kpkt": kpkt, "binning": 128.0 * acts, "finish": 640.0 * acts}


def vpkt_byte_model(vwork, traces, nions_total):
    """Virtual packets (vpkt.cc:76-406) with the same per-unit figures: a 104-byte spawn record per trace, a cell
    step (168 B + kappa: 8 B per ion) per segment, 64 B per line whose opacity is added, 88 B per active bf
    continuum, and the three vstokes read-modify-writes (48 B) of an escaped virtual packet."""
    return (104.0 * traces + (168.0 + 8.0 * nions_total) * vwork["segments"] + 64.0 * vwork["lines"]
            + 88.0 * vwork["bf_active"] + 48.0 * vwork["escaped"])


WORK_NAMES = ["active", "rpkt_steps", "lines_scanned", "line_taus", "kappa_evals", "bf_active", "est_segments",
              "gc_updates", "ma_jumps", "ma_trans", "kpkt", "kpkt_terms", "escaped", "es_scat", "bb_events",
              "cont_events"]

# rocprof names (prefixes) of each class's kernel: k_ma's instance is k_ma<waves, coop, level> (row mode
# k_ma<1, false, false>), k_vpkt's k_vpkt<prefetch, waves>
KERNEL_NAME = {"rpkt": "k_rpkt<2", "ma": "k_ma<", "kpkt": "k_kpkt", "vpkt": "k_vpkt<", "binning": "k_ma_scatter",
               "finish": "k_ma_finish"}


def cpu_share():
    """Threads this process may run on: affinity mask, capped by the cgroup v2 CPU quota; plus host facts."""
    n = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = max(1, int(float(q) / float(per)))
    except (OSError, ValueError):
        pass
    threads = min(n, quota) if quota else n
    model = ""
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                model = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return threads, {"nproc": os.cpu_count(), "affinity": n, "cgroup_quota_cpus": quota, "cpu_model": model}


def _free_port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def self_launch(n, argv):
    """Start n rank processes of this script (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* as torch.distributed.run
    sets them, rendezvous on 127.0.0.1), wait for all of them and return the exit status.  Called before anything
    initialises the GPU: the children are new processes, nothing is exec'd in place.  If one rank fails the others
    are stopped, so a failed rank cannot leave its peers waiting in a barrier."""
    import subprocess

    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    status = 0
    pending = set(range(n))
    while pending:
        for r in list(pending):
            rc = procs[r].poll()
            if rc is None:
                continue
            pending.discard(r)
            if rc != 0 and status == 0:
                status = rc if rc > 0 else 1
                for q in pending:
                    procs[q].terminate()
        time.sleep(0.05)
    return status


def dry_launch(world, rank):
    """Rank bring-up without a GPU: join the gloo group, gather the ranks, rank 0 prints them."""
    if os.environ.get("BENCH_DRY_FAIL_RANK") == str(rank):  # launcher test: a rank that dies before the rendezvous
        sys.exit(3)
    import torch
    import torch.distributed as dist

    dist.init_process_group("gloo")
    got = [None] * world
    dist.all_gather_object(got, {"rank": rank, "local_rank": int(os.environ.get("LOCAL_RANK", "0")), "pid": os.getpid()})
    if rank == 0:
        print(json.dumps({"dry_launch": True, "world": world, "ranks": got}), flush=True)
    dist.destroy_process_group()
    del torch


def ceiling(alg, P, value):
    """The workload's own bound: algorithmic bytes per packet-timestep (every kernel class, SURVEY §8(d) figures)
    and the packet-timesteps/s they allow at the 8 TB/s HBM peak; value as a fraction of it."""
    per = sum(alg.values()) / max(P, 1)
    lim = HBM_PEAK_GBS * 1e9 / max(per, 1e-300)
    return {"alg_bytes_per_packet_timestep": per, "packets_per_s_at_hbm_peak": lim, "frac": value / lim,
            "note": "the 1e8 packets/s/GPU target needs <= 80 KB per packet-timestep at 8 TB/s; this workload's "
                    "macro-atom walks (jumps per packet in work_per_packet) set its bytes"}


def timed_workload(m, P, nts, rank, steps, params=None, etot=None, seed=3000):
    """P resident r-packets of model m at timestep nts, timed like the main line (restore, zero, upload_cellstate
    with the per-cell precompute, transport): one warm step, then `steps` timed ones.  Packets/s, the kernel times,
    the dominant kernel's roofline fraction (engine byte model) and the workload ceiling."""
    from artis_amd import Engine

    m.set_timestep(nts)
    prm = ffi_params(m) if params is None else params
    prm.rank = rank
    pk = m.init_rpackets(nts, P, seed=seed + rank, **({} if etot is None else {"etot": etot}))
    eng = Engine(m, params=prm)
    eng.upload_cellstate(nts)
    eng.upload(pk)
    eng.snapshot()
    del pk
    ms, kts, pre, work = [], [], [], np.zeros(16, dtype=np.int64)
    for k in range(steps + 1):
        eng.restore()
        eng.zero_estimators()
        t = time.perf_counter()
        eng.upload_cellstate(nts)
        eng.step_resident(nts, my_rank=rank)
        dt = time.perf_counter() - t
        if k > 0:  # the first step warms up
            ms.append(dt * 1e3)
            kts.append(eng.last_kernel_class_times())
            pre.append(eng.last_precompute_ms())
            work[:] = eng.last_work()
    tables = eng.table_info()
    eng.close()
    alg = byte_model(work, m.nions_total)
    kt = {c: (float(np.mean([t[c][0] for t in kts])), float(np.mean([t[c][1] for t in kts])))
          for c in kts[0]}
    # the dominant kernel class over every class of the step (class_roofline: each class's fraction)
    dom = max((c for c in kt if c in alg), key=lambda c: kt[c][0])
    launches = max(kt[dom][1], 1.)
    gbs = alg[dom] / launches / max(kt[dom][0] / 1e3 / launches, 1e-12) / 1e9
    value = P / (float(np.mean(ms)) / 1e3)
    step_ms = float(np.mean(ms))
    return {"npts_model": m.npts_model, "levels": m.nlevels_total, "lines": m.nlines, "bf_continua": m.nbfcontinua,
            "packets": P, "timestep": nts, "steps": steps, "ms_per_step": step_ms, "value": value,
            "unit": "packets/s", "precompute_ms": float(np.mean(pre)), "kernel_ms": {c: v[0] for c, v in kt.items()},
            "kernel_share_of_step": {c: v[0] / step_ms for c, v in kt.items()},
            "roofline": {"kernel": KERNEL_NAME[dom], "achieved": gbs, "peak": HBM_PEAK_GBS, "frac": gbs / HBM_PEAK_GBS},
            "class_roofline": class_roofline(alg, kt),
            "ceiling": ceiling(alg, P, value),
            "work_per_packet": {k: float(v) / max(P, 1) for k, v in zip(WORK_NAMES, work)}, "tables": tables}


def class_roofline(alg, kt):
    """Per kernel class with a byte model: algorithmic bytes per launch, average launch ms and the HBM fraction."""
    out = {}
    for c, (ms, nl) in kt.items():
        if c not in alg or ms <= 0:
            continue
        nl = max(nl, 1.)
        out[c] = {"alg_bytes_per_launch": alg[c] / nl, "avg_launch_ms": ms / nl,
                  "frac": alg[c] / nl / (ms / nl / 1e3) / 1e9 / HBM_PEAK_GBS}
    return out


def find_traffic(src_sha, P, ngrid, nts, vpkt, kernel_prefix):
    """Measured HBM bytes per launch of the kernel named kernel_prefix from a PMC summary (profiles/pmc_*.json,
    tools/pmc_summary.py: FETCH_SIZE x2 + WRITE_SIZE) made from the same engine sources and workload; (bytes, file)."""
    traffic, src = None, None
    for prof in sorted(glob.glob(os.path.join(REPO, "profiles", "pmc_*.json"))):
        try:
            pm = json.load(open(prof))
        except Exception:
            continue
        if (pm.get("engine_src_sha") == src_sha and pm.get("packets") == P and pm.get("ngrid") == ngrid
                and pm.get("nts") == nts and pm.get("vpkt", 0) == vpkt):
            kd = next((v for k, v in pm.get("kernels", {}).items() if k.startswith(kernel_prefix)), None)
            if kd:
                traffic = kd["hbm_bytes_per_launch"]
                src = os.path.relpath(prof, REPO)
    return traffic, src


def traffic_fields(traffic, src, alg_per_launch, launch_ms):
    """The roofline fields the PMC traffic gives: the fraction of peak by measured bytes beside the byte model's."""
    if traffic is None:
        return {"traffic": None, "traffic_profile": None, "frac_by_traffic": None, "traffic_over_alg": None}
    return {"traffic": traffic, "traffic_profile": src,
            "frac_by_traffic": traffic / max(launch_ms / 1e3, 1e-12) / 1e9 / HBM_PEAK_GBS,
            "traffic_over_alg": traffic / max(alg_per_launch, 1e-300)}


def ffi_params(m):
    from artis_amd import ffi

    return ffi.RunParams.from_buffer_copy(m.params)


def survey_sized_workload(P, steps, nts, rank, progress):
    """SURVEY §8(d)'s specified atom size beside the heavier default: ~100 levels per non-top ion (all level pairs
    joined by a line: 44 550 lines), 56 ionising levels (504 continua), the same 50^3 grid, timestep and P packets
    per GPU, timed like the main line (resident packets, per-step precompute + transport)."""
    from artis_amd.model import Model

    m = Model(ngrid_1d=50, nlevels_per_ion=100, line_window=100, n_resonance=5, n_ionising=56)
    out = timed_workload(m, P, nts, rank, steps)
    out["levels_per_ion"] = 100
    out["macro_atom_jumps_per_packet"] = out["work_per_packet"]["ma_jumps"]
    progress(f"SURVEY-sized workload: {out['ms_per_step']:.0f} ms per step")
    m.close()
    return out


def baseline_configs(P, rank, progress, which=("w7_100_shells", "nebular_onezone", "kilonova")):
    """BASELINE.json configs 2-4 at their stated per-GPU sizes, each timed like the main line (synthetic atomic
    data; the reference's own model / input files where the config names them):
      config 2: classic LTE, 1D 100-shell W7-like model on the 50^3 cuboid, 1e7 r-packets;
      config 3: tests/nebularonezone_inputfiles with the nebular options (NLTE populations, NO_LUT photoionisation
                integrals, binned radiation field, detailed bf estimators, NT), 1e7 packets in its one zone;
      config 4: tests/kilonova_inputfiles (25 shells, relativistic Doppler, excitation temperature T_e), the
                1.25e7-packet per-GPU share of 1e8 on 8 GPUs."""
    from artis_amd.model import Model

    ref = os.path.join(REPO, "tests", "golden", "ref_inputs")

    def files(name):
        d = os.path.join(ref, name)
        mf = os.path.join(d, "model.txt.xz" if os.path.exists(os.path.join(d, "model.txt.xz")) else "model.txt")
        return (os.path.join(d, "input-newrun.txt"), mf, os.path.join(d, "abundances.txt"))

    out = {}
    for name in which:
        if name == "w7_100_shells":
            m, nts, n = Model(ngrid_1d=50, nshells_1d=100), 10, P
        elif name == "nebular_onezone":
            m, nts, n = Model(files=files("nebularonezone"), ngrid_1d=50, nebular=1), 6, P
        else:
            m, nts, n = Model(files=files("kilonova"), ngrid_1d=50, relativistic=1, excitation_te=1), 6, P * 5 // 4
        rec = timed_workload(m, n, nts, rank, 1)
        rec["config"] = {"w7_100_shells": 2, "nebular_onezone": 3, "kilonova": 4}[name]
        out[name] = rec
        progress(f"config {name}: {rec['ms_per_step']:.0f} ms per step, {rec['value']:.3g} packets/s")
        m.close()
    return out


def vpkt_config5(rank, progress, P=10_000_000, nts=30, nobs=4, ngrid=50):
    """BASELINE config 5 (3D 50^3 grid, virtual packets + polarisation, vpkt.cc:76-406, 837-896) at 1e7 packets on one
    GPU, the same workload as `bench.py --vpkt 4 --nts 30` (so its PMC summary applies); the 1e9-packet run's per-GPU
    share of 1.25e8 packets is that command with --packets 125000000.  One warm step, one timed step, timed like the
    main line; the dominant kernel (k_vpkt) with its roofline fraction by the byte model and by measured traffic."""
    from artis_amd import Engine, engine_src_sha, ffi
    from artis_amd.model import Model

    m = Model(ngrid_1d=ngrid)
    m.set_timestep(nts)
    prm = ffi_params(m)
    prm.rank = rank
    pk = m.init_rpackets(nts, P, seed=1000 + rank)
    eng = Engine(m, params=prm)
    vcfg = ffi.VpktConfig(nz_obs=tuple(np.linspace(-0.9, 0.9, nobs)), phi_obs_deg=tuple(np.linspace(0.0, 300.0, nobs)),
                          exclude=(0.0, -1.0, -2.0, 26.0), nprocs=1)
    eng.vpkt_init(vcfg)
    eng.upload_cellstate(nts)
    eng.upload(pk)
    eng.snapshot()
    del pk
    ms, kts, vst, vwk, rnd, work = [], [], [], [], [], np.zeros(16, dtype=np.int64)
    for k in range(2):
        eng.restore()
        eng.zero_estimators()
        t = time.perf_counter()
        eng.upload_cellstate(nts)
        eng.step_resident(nts, my_rank=rank)
        dt = time.perf_counter() - t
        if k > 0:
            ms.append(dt * 1e3)
            kts.append(eng.last_kernel_class_times())
            vst.append(eng.vpkt_last_stats())
            vwk.append(eng.vpkt_last_work())
            rnd.append(eng.last_rounds())
            work[:] = eng.last_work()
    eng.close()
    alg = byte_model(work, m.nions_total)
    ntr = float(np.mean([v[2] for v in vst]))
    vw = {k: float(np.mean([w[k] for w in vwk])) for k in vwk[0]}
    alg["vpkt"] = vpkt_byte_model(vw, ntr, m.nions_total)
    kt = {c: (float(np.mean([t[c][0] for t in kts])), float(np.mean([t[c][1] for t in kts]))) for c in kts[0]}
    kt["vpkt"] = (float(np.mean([v[0] for v in vst])), float(max(np.mean(rnd), 1)))
    dom = max((c for c in kt if c in alg), key=lambda c: kt[c][0])
    launches = max(kt[dom][1], 1.)
    per_launch = alg[dom] / launches
    launch_ms = kt[dom][0] / launches
    gbs = per_launch / max(launch_ms / 1e3, 1e-12) / 1e9
    traffic, src = find_traffic(engine_src_sha(), P, ngrid, nts, nobs, KERNEL_NAME[dom])
    step_ms = float(np.mean(ms))
    out = {"config": 5, "packets": P, "timestep": nts, "observers": nobs, "spectra": int(vcfg.nspectra),
           "ms_per_step": step_ms, "value": P / (step_ms / 1e3), "unit": "packets/s",
           "kernel_ms": {c: v[0] for c, v in kt.items()}, "kernel_share_of_step": {c: v[0] / step_ms for c, v in kt.items()},
           "vpkt": {"ms": kt["vpkt"][0], "traces": int(ntr), "traces_per_s": ntr / max(kt["vpkt"][0] / 1e3, 1e-12),
                    "work_per_trace": {k: v / max(ntr, 1.) for k, v in vw.items()}},
           "roofline": {"kernel": KERNEL_NAME[dom], "achieved": gbs, "peak": HBM_PEAK_GBS, "frac": gbs / HBM_PEAK_GBS,
                        "alg_bytes_per_launch": per_launch, "avg_launch_ms": launch_ms,
                        **traffic_fields(traffic, src, per_launch, launch_ms)},
           "note": "the 1e9-packet config runs 1.25e8 packets per GPU on 8 GPUs: `bench.py --vpkt 4 --nts 30 --packets "
                   "125000000` (profiles/*_bench_vpkt_125M.json)"}
    progress(f"config 5 shape (vpkt, {P} packets): {step_ms:.0f} ms per step")
    m.close()
    return out


def allreduce_cost(eng, rank, iters=20):
    """SURVEY §8(d) 'with and without the RCCL all-reduce' at world size 1: the packed estimator block's size and the
    time of the engine's all-reduce path (block gathered from the estimator arrays, ncclAllReduce, scalars averaged,
    block scattered back) on a one-rank communicator; the xGMI term of N ranks is bounded from the block size."""
    import torch
    from artis_amd import comm_unique_id

    eng.comm_init(0, 1, comm_unique_id())
    eng.allreduce_estimators()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        eng.allreduce_estimators()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) / iters * 1e3
    nbytes = 8 * eng.estimator_block_doubles()
    # ring all-reduce over 8 ranks: every rank sends and receives 2 (N-1)/N of the block; one xGMI link ~153 GB/s
    # (MI355X_MICROARCH.md) as the per-rank bound of one ring
    ring8_ms = 2 * 7 / 8 * nbytes / 153e9 * 1e3
    return {"block_bytes": nbytes, "world1_ms": ms, "ring8_one_link_bound_ms": ring8_ms,
            "note": "world size 1: the gather / scatter of the block around the collective; ring8 bound: the data an "
                    "8-rank ring moves per rank over one 153 GB/s xGMI link"}


def level_mode_workload(rank, progress, P=1_000_000, nts=10):
    """The macro-atom key records in level mode: the 50^3 grid with 5x the bench's lines (line window 160:
    470 745 lines), whose whole-cell records do not fit the HBM budget, so records are kept per (cell, level) pair for
    the pairs the walks use most; P packets per GPU, timed like the main line after one warm step (the placement of
    the first transport is made from the walks of that step)."""
    from artis_amd.model import Model

    # (the generator caps the line count at 100 000 unless told otherwise: the 5x atom needs the cap lifted)
    m = Model(ngrid_1d=50, line_window=160, max_lines=1_000_000)
    out = timed_workload(m, P, nts, rank, 1)
    out["line_window"] = 160
    out["level_mode"] = bool(out["tables"].get("ma_level_records", 0) > 0)
    progress(f"level-mode workload (5x lines, {P} packets): {out['ms_per_step']:.0f} ms per step")
    m.close()
    return out


def timestep_loop(P, nts0, nsteps, rank, progress):
    """The whole do_timestep body on the device (artis_amd.timestep.LteTimestepLoop, sn3d.cc:514-673): update_grid's
    preparation + temperature solution from the previous step's raw estimators (GPU), upload_cellstate (per-cell
    precompute), update_packets on the resident packets, over consecutive timesteps of the bench model; packet
    energies normalised to the cell state's radiation field so the estimators feed update_grid consistently."""
    from artis_amd import Engine
    from artis_amd.model import Model
    from artis_amd.timestep import LteTimestepLoop

    m = Model(ngrid_1d=50)
    m.set_timestep(nts0)
    prm = ffi_params(m)
    prm.rank = rank
    eng = Engine(m, params=prm)
    loop = LteTimestepLoop(m, eng, rank=rank)
    pk = m.init_rpackets(nts0, P, seed=4000 + rank, etot=loop.radiation_energy(nts0))
    eng.upload(pk)
    del pk
    t = time.perf_counter()
    recs = loop.run(nts0, nsteps, progress=progress)
    total = time.perf_counter() - t
    eng.close()
    m.close()
    active = P * nsteps
    return {"packets": P, "timesteps": [r["nts"] for r in recs], "wall_s": total,
            "value": active / total, "unit": "packet-timesteps/s (each packet propagated through every timestep)",
            "per_timestep": recs,
            "note": "timestep k > 0: update_grid (GPU preparation + solution, host cell-state write) -> "
                    "upload_cellstate -> update_packets (resident) -> raw estimators D2H"}


def nebular_update_grid(rank, cpu, progress):
    """SURVEY §8(f) row 4 for the nebular options (artis_gpu_update_grid_nlte): update_grid of BASELINE config 3's
    nebularonezone inputs and of every cell of a 136-cell synthetic nebular model (each with its Spencer-Fano solution),
    from the raw estimators of a GPU transport step; the oracle on the same inputs for the CPU time and parity."""
    from artis_amd import Engine, ffi
    from artis_amd.model import Model

    ref = os.path.join(REPO, "tests", "golden", "ref_inputs", "nebularonezone")
    out = {}
    cases = {
        "onezone": dict(files=(os.path.join(ref, "input-newrun.txt"), os.path.join(ref, "model.txt"),
                               os.path.join(ref, "abundances.txt")), ngrid_1d=10, nlevels_per_ion=30, n_ionising=10,
                        max_lines=2000, nebular=1, nlte_level_max=12, ionpot_scale=0.5),
        "synthetic_136_cells": dict(ngrid_1d=6, nlevels_per_ion=30, n_ionising=10, max_lines=2000, ntstep=20, nebular=1,
                                    nlte_level_max=12, tmin_days=100., tmax_days=300., T0=6000., ionpot_scale=0.5),
    }
    for name, kw in cases.items():
        m = Model(**kw)
        nts = 6 if name == "onezone" else 12
        p = ffi.RunParams.from_buffer_copy(m.params)
        eng = Engine(m, params=p)
        m.set_timestep(nts - 1)
        eng.upload_cellstate(nts - 1)
        est = eng.update_packets(nts - 1, m.init_rpackets(nts - 1, 20000 if name == "onezone" else 8000, seed=5))
        m.set_timestep(nts)
        nt = ffi.NtDataHandle(m)
        arr = ffi.NlteArrays(m, nts, est=est, dep_scale=3e-4 if name == "onezone" else 1.0, seed=12)
        arr.params.num_lte_timesteps = 4 if name == "onezone" else 2
        eng.update_grid_nlte(nt, arr.copy())  # warm
        ag = arr.copy()
        ms = eng.update_grid_nlte(nt, ag)
        eng.close()
        cells = arr.mgi_list
        rec = {"cells": int(len(cells)), "timestep": nts, "gpu_ms": ms, "passes_max": int(ag.iters[cells].max()),
               "spencer_fano_sfpts": 4096}
        if cpu:
            sys.path.insert(0, os.path.join(REPO, "tests"))
            import oracle_lib

            nthreads, _ = cpu_share()
            sub = arr.copy()
            sub.mgi_list = cells[:: max(1, len(cells) // 8)][:8].copy()
            t = time.perf_counter()
            oracle_lib.update_grid_nlte(m, nt, sub, params=p, nthreads=nthreads)
            dt = time.perf_counter() - t
            g = sub.mgi_list
            rec["cpu_baseline"] = {"cells": int(len(g)), "seconds": dt, "threads": nthreads, "kind": "port",
                                   "cells_per_s": len(g) / dt}
            rec["gpu_cells_per_s"] = len(cells) / (ms / 1e3)
            rec["parity_sample"] = {"cells": int(len(g)),
                                    "max_Te_rel": float(np.max(np.abs(ag.Te[g] - sub.Te[g]) / sub.Te[g])),
                                    "max_nne_rel": float(np.max(np.abs(ag.nne[g] - sub.nne[g]) / sub.nne[g])),
                                    "passes_equal": float(np.mean(ag.iters[g] == sub.iters[g]))}
        out[name] = rec
        progress(f"nebular update_grid {name}: {ms:.0f} ms")
        m.close()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--packets", type=int, default=10_000_000, help="packets per GPU (SURVEY.md §8(d): 1e7)")
    ap.add_argument("--ngrid", type=int, default=50)
    ap.add_argument("--line-window", type=int, default=None,
                    help="synthetic atom: lines per level (default 22: 93 798 lines; 160: 470 745, 5x)")
    ap.add_argument("--max-lines", type=int, default=None, help="synthetic atom: line cap (default 100 000)")
    ap.add_argument("--nlevels-per-ion", type=int, default=None, help="synthetic atom: levels per ion (default 400)")
    ap.add_argument("--nts", type=int, default=10)
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="target CPU time of the cpu_baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-update-grid", action="store_true",
                    help="skip the update_grid temperature-solution measurement (artis_gpu_solve_temperatures)")
    ap.add_argument("--vpkt", type=int, default=0,
                    help="virtual packets (BASELINE config 5, vpkt.cc) with this many observer directions; the "
                         "timestep must lie in the vspec window [10 d, 30 d] (e.g. --nts 30)")
    ap.add_argument("--no-extra", action="store_true",
                    help="skip the drop-in host-path timing and the SURVEY §8(d)-sized second workload")
    ap.add_argument("--dry-launch", action="store_true",
                    help="bring up the N ranks over gloo without a GPU and print them (tests the launcher)")
    ap.add_argument("--baseline-config", default=None,
                    help="only the BASELINE config sub-lines named (comma-separated: w7_100_shells, nebular_onezone, "
                         "kilonova; level_mode: the 5x-lines atom at min(--packets, 1e6); timestep_loop: update_grid -> "
                         "upload_cellstate -> update_packets over three timesteps; vpkt5: the config-5 shape, 4 observers at timestep 30), "
                         "at --packets per GPU; prints "
                         "them as one JSON line (for per-config profiles)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(self_launch(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if args.dry_launch:
        dry_launch(world, rank)
        return

    import torch
    import torch.distributed as dist

    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a GPU")
    torch.cuda.set_device(local_rank)
    if world > 1:
        dist.init_process_group("gloo")

    from artis_amd import Engine, engine_src_sha
    from artis_amd import dist as adist
    from artis_amd.model import Model

    def progress(msg):  # rank 0, stderr: a long run shows its phases as they finish
        if rank == 0:
            print(f"[bench] {msg}", file=sys.stderr, flush=True)

    if args.baseline_config:
        which = tuple(args.baseline_config.split(","))
        configs = baseline_configs(args.packets, rank, progress,
                                   which=tuple(w for w in which if w not in ("level_mode", "timestep_loop", "vpkt5")))
        if "level_mode" in which:
            configs["level_mode_5x_lines"] = level_mode_workload(rank, progress, P=min(args.packets, 1_000_000))
        if "timestep_loop" in which:
            configs["timestep_loop"] = timestep_loop(args.packets, args.nts, 3, rank, progress)
        if "vpkt5" in which:
            configs["vpkt_config5_shape"] = vpkt_config5(rank, progress, P=args.packets)
        if rank == 0:
            print(json.dumps({"baseline_configs": configs, "engine_src_sha": engine_src_sha()}), flush=True)
        return

    if rank == 0:  # a heartbeat while one long step runs (a 1.25e8-packet virtual-packet step takes minutes)
        import threading

        t_start = time.time()

        def heartbeat():
            while True:
                time.sleep(60)
                print(f"[bench] ... running, {time.time() - t_start:.0f} s", file=sys.stderr, flush=True)

        threading.Thread(target=heartbeat, daemon=True).start()

    atom = {k: v for k, v in (("line_window", args.line_window), ("max_lines", args.max_lines),
                                ("nlevels_per_ion", args.nlevels_per_ion)) if v is not None}
    model = Model(ngrid_1d=args.ngrid, **atom)
    nts = args.nts
    model.set_timestep(nts)
    params = model.params
    params.rank = rank
    P = args.packets
    packets = model.init_rpackets(nts, P, seed=1000 + rank)
    progress(f"model and {P} packets ready")
    eng = Engine(model, device=local_rank, params=params)
    vcfg = None
    if args.vpkt > 0:
        from artis_amd import ffi

        nobs = args.vpkt
        # observers spread in cos(theta) and phi; spectra: all opacity + three with one source removed
        vcfg = ffi.VpktConfig(nz_obs=tuple(np.linspace(-0.9, 0.9, nobs)),
                              phi_obs_deg=tuple(np.linspace(0.0, 300.0, nobs)), exclude=(0.0, -1.0, -2.0, 26.0),
                              nprocs=world)
        eng.vpkt_init(vcfg)
    eng.upload_cellstate(nts)
    eng.upload(packets)
    eng.snapshot()
    tables = eng.table_info()
    progress(f"engine initialised, packets resident; per-cell tables {tables}")

    if world > 1:
        adist.join(eng, rank, world, dist)

    transport_ms = []
    precompute_ms = []
    work = np.zeros(16, dtype=np.int64)
    rounds = []
    ktimes = []
    vstats = []
    vwork = []
    vdrains = []

    def step(record):
        eng.restore()
        eng.zero_estimators()
        eng.upload_cellstate(nts)
        eng.step_resident(nts, my_rank=rank)
        if world > 1:
            adist.allreduce_engine_estimators(eng)
        if record:
            transport_ms.append(eng.last_transport_ms())
            precompute_ms.append(eng.last_precompute_ms())
            work[:] = eng.last_work()
            rounds.append(eng.last_rounds())
            ktimes.append(eng.last_kernel_class_times())
            if vcfg is not None:
                vstats.append(eng.vpkt_last_stats())
                vdrains.append(eng.vpkt_last_drains())
                vwork.append(eng.vpkt_last_work())

    for w in range(args.warmup):
        step(False)
        progress(f"warmup step {w} done: transport {eng.last_transport_ms():.0f} ms")
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(True)
        progress(f"step {k} done: transport {transport_ms[-1]:.0f} ms")
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    tables = eng.table_info()  # with the placement the last timed steps used
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    total_packet_timesteps = world * P * args.steps
    value = total_packet_timesteps / elapsed
    avg_transport_s = float(np.mean(transport_ms)) / 1e3
    alg = byte_model(work, model.nions_total)
    alg_survey = byte_model(work, model.nions_total, probe_bytes=40.0)
    kt = {k: (float(np.mean([t[k][0] for t in ktimes])), float(np.mean([t[k][1] for t in ktimes])))
          for k in ktimes[0]}
    if vcfg is not None:
        ntr = float(np.mean([v[2] for v in vstats]))
        vw = {k: float(np.mean([w[k] for w in vwork])) for k in vwork[0]}
        alg["vpkt"] = alg_survey["vpkt"] = vpkt_byte_model(vw, ntr, model.nions_total)
        kt["vpkt"] = (float(np.mean([v[0] for v in vstats])), float(max(np.mean(rounds), 1)))
    dom = max((k for k in kt if k in alg), key=lambda k: kt[k][0])
    dom_ms, dom_launches = kt[dom]
    launches = max(dom_launches, 1.0)
    bytes_per_launch = alg[dom] / launches
    avg_launch_s = dom_ms / 1e3 / launches
    achieved_gbs = bytes_per_launch / max(avg_launch_s, 1e-12) / 1e9
    achieved_survey = alg_survey[dom] / launches / max(avg_launch_s, 1e-12) / 1e9
    src_sha = engine_src_sha()
    traffic, traffic_src = find_traffic(src_sha, P, args.ngrid, nts, args.vpkt, KERNEL_NAME[dom])
    allreduce = None
    if world == 1 and not args.no_extra:
        allreduce = allreduce_cost(eng, rank)
        progress(f"estimator block all-reduce (world 1): {allreduce['world1_ms']:.2f} ms for "
                 f"{allreduce['block_bytes'] / 1e6:.1f} MB")
    cpu = None
    parity_line = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and vcfg is None:
        sys.path.insert(0, os.path.join(REPO, "tests"))
        import oracle_lib
        import parity

        nthreads, host = cpu_share()
        calib = packets[:256].copy()
        t = time.perf_counter()
        oracle_lib.update_packets(model, nts, calib, nthreads=nthreads)
        rate = 256 / max(time.perf_counter() - t, 1e-6)
        n_sample = int(min(P, max(256, rate * args.cpu_seconds)))
        sample = packets[:n_sample].copy()
        t = time.perf_counter()
        oracle_lib.update_packets(model, nts, sample, nthreads=nthreads)
        cpu_dt = time.perf_counter() - t
        # parity on the same sample: the engine's packets after the timed steps are the same histories
        gpu_pk = np.zeros_like(packets)
        eng.download(gpu_pk)
        gs = gpu_pk[:n_sample]
        bad = parity.discrete_mismatch(gs, sample)
        # the CPU-vs-CPU noise floor: the same sample size from a different seed through the oracle
        # (the same energy per packet as the engine's ensemble: etot scaled to the sample's share)
        other = model.init_rpackets(nts, n_sample, seed=2000 + rank, etot=1e45 * n_sample / P)
        oracle_lib.update_packets(model, nts, other, nthreads=nthreads)
        lum = lambda pk: float(pk["e_rf"][pk["type"] == 32].sum())  # noqa: E731  escaped luminosity of the step
        parity_line = {
            "sample_packets": n_sample,
            "discrete_state_match": float(1.0 - bad.mean()),
            "max_fp_rel": max(parity.fp_max_rel(gs, sample, ~bad).values()),
            "spectrum_l1": parity.spectrum_l1(gs, sample),
            "spectrum_l1_100bin": float(np.abs(parity.spectrum(gs, 100) - parity.spectrum(sample, 100)).sum() /
                                        max(parity.spectrum(sample, 100).sum(), 1e-300)),
            "lightcurve_l1": abs(lum(gs) - lum(sample)) / max(lum(sample), 1e-300),
            "cpu_two_seed_floor": {
                "spectrum_l1": parity.spectrum_l1(other, sample),
                "spectrum_l1_100bin": float(np.abs(parity.spectrum(other, 100) - parity.spectrum(sample, 100)).sum() /
                                            max(parity.spectrum(sample, 100).sum(), 1e-300)),
                "lightcurve_l1": abs(lum(other) - lum(sample)) / max(lum(sample), 1e-300),
                "seeds": "ensemble seeds 1000+rank (the GPU's) and 2000+rank, same sample size, both on the oracle"},
            "spectrum": "escaped-packet energy in 1000 (and 100) log bins of nu_rf over [NU_MIN_R, NU_MAX_R] "
                        "(spec.out binning) for the one timestep; light curve: the step's escaped luminosity",
        }
        cpu = {
            "value": n_sample / cpu_dt,
            "unit": "packets/s",
            "cores": nthreads,
            "host": host,
            "kind": "port",
            "sample": f"first {n_sample} packets of the same ensemble, same timestep, {cpu_dt:.1f} s",
        }

    dropin = None
    if rank == 0 and vcfg is None and not args.no_extra:
        # INTEGRATION.md's drop-in call: artis_gpu_update_packets on host AoS packets (H2D, AoS->SoA, transport,
        # SoA->AoS, D2H, estimators added into host arrays) -- the resident path's transport plus the PCIe round trip
        tms = []
        for k in range(2):
            host = packets.copy()
            est_h = model.new_estimators()
            t = time.perf_counter()
            eng.update_packets(nts, host, est_h, my_rank=rank)
            dt = time.perf_counter() - t
            if k > 0:
                tms.append((dt * 1e3, eng.last_transport_ms()))
            del host
        dropin = {"ms_per_step": tms[-1][0], "value": P / (tms[-1][0] / 1e3), "unit": "packets/s",
                  "transport_ms": tms[-1][1], "host_transfer_ms": tms[-1][0] - tms[-1][1],
                  "bytes_each_way": int(P) * 304,
                  "note": "packets on the host in the reference's 304-byte layout; cell precompute not included "
                          "(the cell state was uploaded once, as in the reference's loop)"}
        progress(f"drop-in host path: {dropin['ms_per_step']:.0f} ms per step")

    ugrid = None
    if rank == 0 and not args.no_update_grid and vcfg is None:
        # SURVEY §8(f) row 4, after the timed region: update_grid's temperature / ionisation solution for every
        # non-empty cell (artis_gpu_solve_temperatures), and the oracle on a cell sample for the CPU rate and parity
        from artis_amd import ffi

        t_cur = 1.5 * float(model.cfg.tmin_days) * 86400.0
        te = ffi.TeArrays(model, t_current=t_cur, seed=4)
        eng.solve_temperatures(te.copy())  # warm
        te_ms = eng.solve_temperatures(te)
        ugrid = {"kernel": "k_te_bfheat + k_te_solve", "cells": int(len(te.mgi_list)), "gpu_ms": te_ms,
                 "rooted_cells": int((te.iters[te.mgi_list] > 0).sum())}
        if not args.no_cpu_baseline:
            sys.path.insert(0, os.path.join(REPO, "tests"))
            import oracle_lib

            nthreads, _ = cpu_share()
            sub = ffi.TeArrays(model, t_current=t_cur, seed=4)
            sub.mgi_list = te.mgi_list[:: max(1, len(te.mgi_list) // 128)][:128].copy()
            t = time.perf_counter()
            oracle_lib.solve_temperatures(model, sub, nthreads=nthreads)
            dt = time.perf_counter() - t
            g = sub.mgi_list
            agree = (sub.iters[g] == te.iters[g]) & (np.abs(sub.Te[g] - te.Te[g]) <= 1e-9 * np.abs(sub.Te[g]))
            ugrid["cpu_baseline"] = {"cells": int(len(g)), "seconds": dt, "threads": nthreads, "kind": "port",
                                     "cells_per_s": len(g) / dt}
            ugrid["gpu_cells_per_s"] = len(te.mgi_list) / (te_ms / 1e3)
            ugrid["parity_sample"] = {"cells": int(len(g)), "iterations_and_Te_agree": float(agree.mean())}

    eng.close()
    neb = None
    if rank == 0 and not args.no_update_grid and vcfg is None:
        neb = nebular_update_grid(rank, not args.no_cpu_baseline, progress)
    survey8d = configs = tloop = lvl = None
    if rank == 0 and world == 1 and vcfg is None and not args.no_extra:
        survey8d = survey_sized_workload(P, 2, nts, rank, progress)
        configs = baseline_configs(P, rank, progress)
        tloop = timestep_loop(P, nts, 3, rank, progress)
        lvl = level_mode_workload(rank, progress)
        configs["vpkt_config5_shape"] = vpkt_config5(rank, progress)

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "packets/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {
                "workload": (f"synthetic 3D {args.ngrid}^3 uniform-grid model (ARTIS model_type 3), Fe/Co/Ni II-V "
                             f"{model.nlevels_total} levels, {model.nlines} lines, {model.nbfcontinua} bf continua; "
                             f"pure r-packet ensemble advanced through timestep {nts} (macro-atom + k-packet "
                             f"closure, LTE classic options)"),
                "packets_per_gpu": P,
                "grid": f"{args.ngrid}^3",
                "timestep": nts,
                "parallelism": (f"packet-sharded x{world}, engine RCCL all-reduce of the estimator block"
                                if world > 1 else "1 GPU"),
            },
            "roofline": {
                "bound": "hbm",
                "achieved": achieved_gbs,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved_gbs / HBM_PEAK_GBS,
                **traffic_fields(traffic, traffic_src, bytes_per_launch, avg_launch_s * 1e3),
                "engine_src_sha": src_sha,
                "kernel": KERNEL_NAME[dom],
                "achieved_survey_model": achieved_survey,
                "frac_survey_model": achieved_survey / HBM_PEAK_GBS,
                "alg_bytes_per_launch": bytes_per_launch,
                "avg_launch_ms": avg_launch_s * 1e3,
                "launches_per_step": launches,
                "transport_alg_GBps": sum(alg.values()) / avg_transport_s / 1e9,
            },
            "cpu_baseline": cpu,
            "parity_vs_cpu": parity_line,
            "precompute_ms": float(np.mean(precompute_ms)),
            "transport_ms": float(np.mean(transport_ms)),
            "event_rounds": int(np.max(rounds)) if rounds else 0,
            "kernel_ms": {k: v[0] for k, v in kt.items()},
            "other_kernels_ms": float(np.mean([sum(t[c][0] for c in ("classify", "binning", "exact", "finish"))
                                               for t in ktimes])),
            "kernel_roofline": class_roofline(alg, kt),
            "ma_ps_per_jump": kt["ma"][0] * 1e9 / max(float(work[8]), 1.0),
            "work_per_packet": {k: float(v) / max(P, 1) for k, v in zip(WORK_NAMES, work)},
            "ceiling": ceiling(alg, P, value / world),
        }
        if allreduce is not None:
            line["estimator_allreduce"] = allreduce
        if ugrid is not None:
            line["update_grid"] = ugrid
        if neb is not None:
            line["update_grid_nebular"] = neb
        if dropin is not None:
            line["dropin_host_path"] = dropin
        if survey8d is not None:
            line["workload_survey_8d"] = survey8d
        if configs is not None:
            line["baseline_configs"] = configs
        if tloop is not None:
            line["timestep_loop"] = tloop
        if lvl is not None:
            line["level_mode_5x_lines"] = lvl
        if vcfg is not None:
            vms = float(np.mean([v[0] for v in vstats]))
            line["config"]["workload"] += (f"; virtual packets: {vcfg.nobs} observers x {vcfg.nspectra} spectra, "
                                           f"vspec window 10-30 d, 3500-10000 A (vpkt.h defaults)")
            line["vpkt"] = {"ms": vms, "spawns": int(np.mean([v[1] for v in vstats])),
                            "traces": int(np.mean([v[2] for v in vstats])),
                            "traces_per_s": float(np.mean([v[2] for v in vstats])) / max(vms / 1e3, 1e-12),
                            "buffer_drains": int(np.max(vdrains))}
            ntr = max(line["vpkt"]["traces"], 1)
            line["vpkt"]["work_per_trace"] = {k: float(np.mean([w[k] for w in vwork])) / ntr for k in vwork[0]}
        line["tables"] = tables
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
