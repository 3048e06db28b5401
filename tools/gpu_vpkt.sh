#!/bin/bash
# Virtual-packet parity tests + the vpkt bench (BASELINE config 5 shape) at 1e6 and 1e7 packets.
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_vpkt.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/gpu_vpkt_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --nts 30 --vpkt 4 --packets 1000000 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/vpkt1m.json 2> gpurun_out/vpkt1m.err &&
timeout -k 10 400 python -u bench.py --nts 30 --vpkt 4 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/vpkt10m.json 2> gpurun_out/vpkt10m.err
