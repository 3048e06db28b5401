#!/bin/bash
# Diagnostics: wave statistics of the bench step, the virtual-packet bench, and an A/B of k_ma occupancy.
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
ARTIS_GPU_STATS=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/stats.json 2> gpurun_out/stats.err &&
timeout -k 10 300 python -u bench.py --nts 30 --vpkt 4 --packets 1000000 --steps 1 --warmup 1 > gpurun_out/vpkt1m.json 2> gpurun_out/vpkt1m.err &&
timeout -k 10 400 python -u bench.py --nts 30 --vpkt 4 --steps 1 --warmup 1 > gpurun_out/vpkt10m.json 2> gpurun_out/vpkt10m.err &&
timeout -k 10 300 python -u bench.py --nts 30 --packets 10000000 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/nts30.json 2> gpurun_out/nts30.err &&
P=10000000 timeout -k 10 600 bash tools/ab_bench.sh ARTIS_GPU_MA_OCC=1 ARTIS_GPU_MA_OCC=8 > gpurun_out/ab_occ.txt 2>&1
