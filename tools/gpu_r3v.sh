#!/bin/bash
# round 3v: the 1.25e8-packet config-5 share (virtual packets, 4 observers, timestep 30) on the final engine
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 1100 python -u bench.py --packets 125000000 --vpkt 4 --nts 30 --steps 1 --warmup 1 --no-cpu-baseline \
  --no-update-grid --no-extra > gpurun_out/r3v_bench_vpkt_125M.json 2> gpurun_out/r3v_bench_vpkt_125M.err
rc=$?; tail -4 gpurun_out/r3v_bench_vpkt_125M.err; exit $rc
