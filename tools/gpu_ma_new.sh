#!/bin/bash
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py tests/test_gpu_gamma.py tests/test_gpu_vpkt.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ma_parity.log 2>&1 || exit 1
P=10000000 timeout -k 10 600 bash tools/ab_bench.sh ARTIS_GPU_MA_OCC=1 ARTIS_GPU_MA_OCC=8 > gpurun_out/ab_ma2.txt 2>&1
