#!/bin/bash
# One GPU call: parity tests, bench line, rocprofv3 kernel stats of the same bench.
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 &&
timeout -k 10 400 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 -u bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err
