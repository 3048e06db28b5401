#!/bin/bash
# One GPU call: (1) the bench line at HEAD, (2) one step with the stamps build (per-phase cycles of the r-packet
# step, ARTIS_GPU_STATS), (3) the config-5 per-GPU share (1.25e8 packets on one MI355X) for one timed step,
# (4) the FETCH/WRITE counter passes of the default bench configuration (1e7 packets).
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
timeout -k 10 300 python3 -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err &&
ARTIS_GPU_STATS=1 ARTIS_GPU_SO=artis_amd/lib/libartis_gpu_stamps.so timeout -k 10 200 python3 -u bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/stamps.json 2> gpurun_out/stamps.err &&
timeout -k 10 600 python3 -u bench.py --packets 125000000 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/big.json 2> gpurun_out/big.err &&
B="python3 bench.py --packets 10000000 --steps 1 --warmup 0 --no-cpu-baseline" &&
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc/fetch -o run -- $B > gpurun_out/pmc/f.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc/write -o run -- $B > gpurun_out/pmc/w.log 2>&1
