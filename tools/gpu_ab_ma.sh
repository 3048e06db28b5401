#!/bin/bash
# k_ma A/B: record-line touch depth (ARTIS_GPU_MA_TOUCH) and refill threshold (ARTIS_GPU_REFILL) at bench size;
# parity suite under the touch variant first.
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
ARTIS_GPU_MA_TOUCH=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/ab_parity.log 2>&1 || exit 1
P=10000000 timeout -k 10 900 bash tools/ab_bench.sh ARTIS_GPU_MA_TOUCH=0 ARTIS_GPU_MA_TOUCH=1 ARTIS_GPU_MA_TOUCH=2 ARTIS_GPU_MA_TOUCH=3 ARTIS_GPU_MA_TOUCH=5 ARTIS_GPU_REFILL=16 ARTIS_GPU_REFILL=48 > gpurun_out/ab_ma.txt 2>&1
