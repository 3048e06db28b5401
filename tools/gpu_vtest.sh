#!/bin/bash
# the vpkt GPU tests incl. the general-kernel variants
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_vpkt.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/vtest.log 2>&1
rc=$?; tail -4 gpurun_out/vtest.log; exit $rc
