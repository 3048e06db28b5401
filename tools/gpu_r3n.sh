#!/bin/bash
# round 3n: k_ma record-line LDS layout swizzle and chunked key search: parity suite on the in-tree engine, then the
# A/B (r3m: before both; swz: swizzle only; main: swizzle + 8-key chunk search)
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3n_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3n_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 bash tools/gpu_ab_so.sh r3m swz main > gpurun_out/r3n_ab.txt 2>&1
rc=$?; cat gpurun_out/r3n_ab.txt; exit $rc
