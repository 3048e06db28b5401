#!/bin/bash
# round 3q: k_vpkt without the gather walk when every cell has a coefficient row (k_vpkt<0, occ>): vpkt parity
# tests, then the config-5 shape A/B (1e7 packets, timestep 30, 4 observers): default (table-only kernel, 2 waves per
# SIMD), the general kernel (ARTIS_VPKT_LCONLY=0), table-only at 1 and 3 waves
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_vpkt.py tests/test_gpu_ref_inputs.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3q_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3q_tests.log; [ $rc -eq 0 ] || exit $rc
BENCH_ARGS="--nts 30 --vpkt 4" timeout -k 10 1000 bash tools/gpu_ab_so.sh main "main:ARTIS_VPKT_LCONLY=0" "main:ARTIS_VPKT_OCC=1" "main:ARTIS_VPKT_OCC=3" > gpurun_out/r3q_ab.txt 2>&1
rc=$?; cat gpurun_out/r3q_ab.txt; exit $rc
