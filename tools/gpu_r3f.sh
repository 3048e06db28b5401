#!/bin/bash
# round 3f: bounded vpkt spawn buffer -- vpkt parity tests, then the 1.25e8-packet vpkt share
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_vpkt.py -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r3f_vpkt_tests.log 2>&1 || { tail -40 gpurun_out/r3f_vpkt_tests.log; exit 1; }
tail -3 gpurun_out/r3f_vpkt_tests.log
timeout -k 10 1000 python -u bench.py --packets 125000000 --vpkt 4 --nts 30 --steps 1 --warmup 1 \
  > gpurun_out/r3f_bench_vpkt_125M.json 2> gpurun_out/r3f_bench_vpkt_125M.err || { tail -20 gpurun_out/r3f_bench_vpkt_125M.err; exit 1; }
tail -4 gpurun_out/r3f_bench_vpkt_125M.err
