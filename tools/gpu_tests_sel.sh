#!/bin/bash
# Selected GPU tests (GPU_TESTS), then optionally a bench line.
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest ${GPU_TESTS:-tests} -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
