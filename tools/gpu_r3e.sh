#!/bin/bash
# round 3e: partial-cache re-placement test, then the 5x-lines model at a small packet count
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -k "budget or partial" \
  > gpurun_out/r3e_parity.log 2>&1 || { tail -40 gpurun_out/r3e_parity.log; exit 1; }
tail -3 gpurun_out/r3e_parity.log
timeout -k 10 500 python -u bench.py --line-window 160 --max-lines 600000 --no-cpu-baseline --no-update-grid --no-extra \
  --packets 100000 --steps 2 --warmup 1 > gpurun_out/r3e_bench_5xlines_1e5.json 2> gpurun_out/r3e_bench_5xlines_1e5.err \
  || { tail -20 gpurun_out/r3e_bench_5xlines_1e5.err; exit 1; }
tail -4 gpurun_out/r3e_bench_5xlines_1e5.err
