#!/bin/bash
# Bench line + rocprofv3 kernel stats of the same bench command (no tests).
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 -u bench.py --no-cpu-baseline > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err
