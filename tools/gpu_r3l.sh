#!/bin/bash
# round 3l: k_ma A/B: two walk slots per lane (k_ma2, default) at 3 and 4 waves per SIMD vs one slot (k_ma<true>),
# each with and without the 3-word metadata load; GPU tests of the parity files first
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ref_inputs.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3l_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3l_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 bash tools/gpu_ab_so.sh "sub:ARTIS_GPU_MA_SLOTS=1 ARTIS_GPU_STATS=1" main "main:ARTIS_GPU_MA2_OCC=4" "main:ARTIS_GPU_MA_SLOTS=1" meta3 "meta3:ARTIS_GPU_MA2_OCC=4" "meta3:ARTIS_GPU_MA_SLOTS=1" > gpurun_out/r3l_ab.txt 2>&1
rc=$?; cat gpurun_out/r3l_ab.txt; exit $rc
