#!/bin/bash
# Full parity suite at the new defaults, k_rpkt occupancy-3 A/B, the bench line, its rocprofv3 kernel stats,
# and the vpkt bench at 1e7 packets.
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 &&
ARTIS_GPU_RPKT_OCC=3 timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_rocc3.json 2> gpurun_out/bench_rocc3.err &&
timeout -k 10 400 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 -u bench.py --no-cpu-baseline > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err &&
timeout -k 10 400 python -u bench.py --nts 30 --vpkt 4 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/vpkt10m.json 2> gpurun_out/vpkt10m.err
