"""bench.py -- packet-timesteps per second of the MI355X update_packets engine on the synthetic 50^3 grid.

python bench.py --gpus N --steps K --warmup W          (N>1: launched by torch.distributed.run, one rank/GPU)

One step = one update_packets(nts) of this rank's P resident packets, all in HBM before timing starts:
  packets reset to the same initial ensemble (device-to-device copy), estimators zeroed, the per-timestep cell
  precompute (artis_gpu_upload_cellstate: cell-state H2D + per-cell table kernels), the transport kernel, and
  for N>1 the RCCL all-reduce of the packed estimator block (radfield J/nuJ, heating/photoionisation
  estimators, line statistics, event counters) -- the reference's mpi_reduce_estimators (sn3d.cc:582).
Packets are sharded: every rank propagates its own full-energy ensemble (rank-specific seed and RNG key), so
per-GPU work is fixed as N grows ("weak").  value = N * P * K / max-over-ranks wall time.

roofline: the dominant kernel class of the event-queue transport (k_ma or k_rpkt): its algorithmic bytes
(SURVEY.md §8(d) per-unit figures over the engine's own event counters, split by the kernel that does the
work) per launch / its average launch time, measured with HIP events around every launch on the engine
stream, against 8.0 TB/s.  traffic: measured HBM bytes per launch of that kernel (rocprofv3 FETCH_SIZE x2 +
WRITE_SIZE, profiles/pmc_*.json) when a PMC summary of the same configuration is committed.
cpu_baseline: the CPU oracle (oracle/liboracle.so, OpenMP) on a bounded sample of the same workload, rank 0
at N=1 only.
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


def byte_model(work, nions_total):
    """SURVEY.md §8(d) algorithmic bytes per kernel class from the work counters (include/artis_constants.h
    enum artis_work): the r-packet kernel reads/writes the record, steps, scans lines, evaluates kappa and
    estimators; the macro-atom kernel reads a 72-byte rate record per jump and 40 bytes per transition touched;
    the k-packet kernel scans cooling terms."""
    w = [float(x) for x in work]
    rpkt = (608.0 * w[0] + 168.0 * w[1] + 64.0 * w[2] + 88.0 * w[5] + 8.0 * nions_total * w[4] + 48.0 * w[6]
            + 32.0 * w[7])
    ma = 72.0 * w[8] + 40.0 * w[9]
    kpkt = 16.0 * w[11]
    return {"rpkt": rpkt, "ma": ma, "kpkt": kpkt}


KERNEL_NAME = {"rpkt": "k_rpkt<2>", "ma": "k_ma<true, 1>", "kpkt": "k_kpkt"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--packets", type=int, default=10_000_000, help="packets per GPU (SURVEY.md §8(d): 1e7)")
    ap.add_argument("--ngrid", type=int, default=50)
    ap.add_argument("--nts", type=int, default=10)
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="target CPU time of the cpu_baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--vpkt", type=int, default=0,
                    help="virtual packets (BASELINE config 5, vpkt.cc) with this many observer directions; the "
                         "timestep must lie in the vspec window [10 d, 30 d] (e.g. --nts 30)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a GPU")
    torch.cuda.set_device(local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    from artis_amd import Engine
    from artis_amd.model import Model

    model = Model(ngrid_1d=args.ngrid)
    nts = args.nts
    model.set_timestep(nts)
    params = model.params
    params.rank = rank
    P = args.packets
    packets = model.init_rpackets(nts, P, seed=1000 + rank)
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

    red = None
    if world > 1:
        red = torch.empty(eng.estimator_block_doubles(), dtype=torch.float64, device="cuda")

    transport_ms = []
    precompute_ms = []
    work = np.zeros(16, dtype=np.int64)
    rounds = []
    ktimes = []
    vstats = []
    vwork = []

    def step(record):
        eng.restore()
        eng.zero_estimators()
        eng.upload_cellstate(nts)
        eng.step_resident(nts, my_rank=rank)
        if red is not None:
            eng.estimator_block_to_device(red.data_ptr())
            dist.all_reduce(red)
            eng.estimator_block_from_device(red.data_ptr())
        if record:
            transport_ms.append(eng.last_transport_ms())
            precompute_ms.append(eng.last_precompute_ms())
            work[:] = eng.last_work()
            rounds.append(eng.last_rounds())
            ktimes.append(eng.last_kernel_times())
            if vcfg is not None:
                vstats.append(eng.vpkt_last_stats())
                vwork.append(eng.vpkt_last_work())

    for _ in range(args.warmup):
        step(False)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    total_packet_timesteps = world * P * args.steps
    value = total_packet_timesteps / elapsed
    avg_transport_s = float(np.mean(transport_ms)) / 1e3
    alg = byte_model(work, model.nions_total)
    kt = {k: (float(np.mean([t[k][0] for t in ktimes])), float(np.mean([t[k][1] for t in ktimes])))
          for k in ("rpkt", "ma", "kpkt")}
    dom = max(("rpkt", "ma"), key=lambda k: kt[k][0])
    dom_ms, dom_launches = kt[dom]
    launches = max(dom_launches, 1.0)
    bytes_per_launch = alg[dom] / launches
    avg_launch_s = dom_ms / 1e3 / launches
    achieved_gbs = bytes_per_launch / max(avg_launch_s, 1e-12) / 1e9
    traffic = None
    for prof in sorted(glob.glob(os.path.join(REPO, "profiles", "pmc_*.json"))):
        try:
            pm = json.load(open(prof))
        except Exception:
            continue
        if pm.get("packets") == P and pm.get("ngrid") == args.ngrid and pm.get("nts") == nts:
            kd = pm.get("kernels", {}).get(KERNEL_NAME[dom])
            if kd:
                traffic = kd["hbm_bytes_per_launch"]
    cpu = None
    parity_line = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and vcfg is None:
        sys.path.insert(0, os.path.join(REPO, "tests"))
        import oracle_lib
        import parity

        nthreads = min(16, os.cpu_count() or 1)
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
        parity_line = {
            "sample_packets": n_sample,
            "discrete_state_match": float(1.0 - bad.mean()),
            "max_fp_rel": max(parity.fp_max_rel(gs, sample, ~bad).values()),
            "spectrum_l1": parity.spectrum_l1(gs, sample),
            "spectrum": "escaped-packet energy in 1000 log bins of nu_rf over [NU_MIN_R, NU_MAX_R] (spec.out binning)",
        }
        cpu = {
            "value": n_sample / cpu_dt,
            "unit": "packets/s",
            "cores": nthreads,
            "kind": "port",
            "sample": f"first {n_sample} packets of the same ensemble, same timestep, {cpu_dt:.1f} s",
        }

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
                "parallelism": f"packet-sharded x{world}, RCCL estimator all-reduce" if world > 1 else "1 GPU",
            },
            "roofline": {
                "bound": "hbm",
                "achieved": achieved_gbs,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved_gbs / HBM_PEAK_GBS,
                "traffic": traffic,
                "kernel": KERNEL_NAME[dom],
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
            "work_per_packet": {k: float(v) / max(P, 1) for k, v in zip(
                ["active", "rpkt_steps", "lines_scanned", "line_taus", "kappa_evals", "bf_active", "est_segments",
                 "gc_updates", "ma_jumps", "ma_trans", "kpkt", "kpkt_terms", "escaped", "es_scat", "bb_events",
                 "cont_events"], work)},
        }
        if vcfg is not None:
            vms = float(np.mean([v[0] for v in vstats]))
            line["config"]["workload"] += (f"; virtual packets: {vcfg.nobs} observers x {vcfg.nspectra} spectra, "
                                           f"vspec window 10-30 d, 3500-10000 A (vpkt.h defaults)")
            line["vpkt"] = {"ms": vms, "spawns": int(np.mean([v[1] for v in vstats])),
                            "traces": int(np.mean([v[2] for v in vstats])),
                            "traces_per_s": float(np.mean([v[2] for v in vstats])) / max(vms / 1e3, 1e-12)}
            ntr = max(line["vpkt"]["traces"], 1)
            line["vpkt"]["work_per_trace"] = {k: float(np.mean([w[k] for w in vwork])) / ntr for k in vwork[0]}
        print(json.dumps(line), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
