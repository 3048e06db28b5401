#!/bin/bash
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ma_parity.log 2>&1 || exit 1
ARTIS_GPU_STATS=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/stats.json 2> gpurun_out/stats.err || exit 1
P=10000000 timeout -k 10 600 bash tools/ab_bench.sh ARTIS_GPU_MA_WAVES=2 ARTIS_GPU_MA_WAVES=3 ARTIS_GPU_MA_WAVES=4 > gpurun_out/ab_ma3.txt 2>&1
