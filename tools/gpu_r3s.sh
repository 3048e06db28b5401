#!/bin/bash
# round 3s: ion-major k_cooling (populations from popsT): GPU parity suite, then the bench A/B against the r3r engine
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3s_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r3s_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 bash tools/gpu_ab_so.sh r3r main r3r main > gpurun_out/r3s_ab.txt 2>&1
rc=$?; cat gpurun_out/r3s_ab.txt; exit $rc
