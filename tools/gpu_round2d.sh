#!/bin/bash
# Round-2d: the update_grid temperature solver on the GPU (parity tests with the default lane groups and with one
# cell per lane for the A/B), then the bench line (incl. update_grid) and its rocprofv3 kernel statistics.
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r2d
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_te_solver.py -x -v -s --timeout 200 --timeout-method thread > $O/te_tests.log 2>&1 &&
ARTIS_GPU_TE_LANES=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_te_solver.py -x -v -s --timeout 200 --timeout-method thread -k bench_grid > $O/te_tests_lanes1.log 2>&1 &&
timeout -k 10 400 python3 -u bench.py > $O/bench.json 2> $O/bench.err &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -u bench.py --no-cpu-baseline > $O/bench_prof.json 2> $O/bench_prof.err
