#!/bin/bash
# rocprofv3 PMC passes over the bench (one counter group per pass, each its own run).
# P (packets, default 1e6) and EXTRA (further bench args) select the configuration.
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
P=${P:-1000000}
B="python3 bench.py --packets $P --steps 1 --warmup 0 --no-cpu-baseline $EXTRA"
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1 || true
timeout -s KILL 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc/fetch -o run -- $B > gpurun_out/pmc/f.log 2>&1 &&
timeout -s KILL 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc/write -o run -- $B > gpurun_out/pmc/w.log 2>&1 &&
timeout -s KILL 600 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -d gpurun_out/pmc/tcc -o run -- $B > gpurun_out/pmc/t.log 2>&1 &&
timeout -s KILL 600 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum --kernel-trace -d gpurun_out/pmc/tcp -o run -- $B > gpurun_out/pmc/p.log 2>&1 &&
timeout -s KILL 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES --kernel-trace -d gpurun_out/pmc/sq -o run -- $B > gpurun_out/pmc/s.log 2>&1
