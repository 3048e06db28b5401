#!/bin/bash
# Round-2c check at HEAD in one GPU call: the full GPU parity suite, the bench line and rocprofv3 kernel statistics
# of the bench.
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r2c
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 &&
timeout -k 10 400 python3 -u bench.py > $O/bench.json 2> $O/bench.err &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -u bench.py --no-cpu-baseline > $O/bench_prof.json 2> $O/bench_prof.err
