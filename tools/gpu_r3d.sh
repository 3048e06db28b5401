#!/bin/bash
# round 3d: table-budget parity, smoke, the default bench line (drop-in + SURVEY-sized extras) and a 5x-lines line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r3d_parity.log 2>&1 || { tail -40 gpurun_out/r3d_parity.log; exit 1; }
tail -3 gpurun_out/r3d_parity.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3d_smoke.log 2>&1 || { tail -20 gpurun_out/r3d_smoke.log; exit 1; }
tail -2 gpurun_out/r3d_smoke.log
timeout -k 10 900 python -u bench.py > gpurun_out/r3d_bench.json 2> gpurun_out/r3d_bench.err || { tail -20 gpurun_out/r3d_bench.err; exit 1; }
tail -3 gpurun_out/r3d_bench.err
timeout -k 10 400 python -u bench.py --line-window 160 --max-lines 600000 --no-cpu-baseline --no-update-grid --no-extra \
  --packets 1000000 --steps 1 --warmup 1 > gpurun_out/r3d_bench_5xlines.json 2> gpurun_out/r3d_bench_5xlines.err || { tail -20 gpurun_out/r3d_bench_5xlines.err; exit 1; }
tail -3 gpurun_out/r3d_bench_5xlines.err
