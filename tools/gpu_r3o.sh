#!/bin/bash
# round 3o: the config-5 shape (virtual packets, 4 observers, timestep 30, 1e7 packets) bench line under rocprofv3
# kernel statistics, at the engine hash of profiles/pmc_r03m_vpkt.json (so the line carries k_vpkt's PMC traffic)
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r3o
mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -u bench.py --packets 10000000 --nts 30 --vpkt 4 --steps 1 --warmup 1 --no-cpu-baseline --no-update-grid --no-extra > $O/bench_vpkt.json 2> $O/bench_vpkt.err
rc=$?; tail -c 1500 $O/bench_vpkt.json; exit $rc
