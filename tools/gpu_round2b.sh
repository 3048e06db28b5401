#!/bin/bash
# Round-2 measurements at HEAD in one GPU call: the full GPU parity suite, the bench line, per-phase cycle stamps
# (diagnostic build), rocprofv3 kernel statistics of the bench, FETCH/WRITE counter passes of the bench
# configuration, a FETCH_SIZE calibration on random 128-byte lines of known byte count (tools/linerate), the
# config-5 shape with virtual packets, and the config-5 per-GPU share (1.25e8 packets).
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r2b
mkdir -p $O/pmc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 &&
timeout -k 10 400 python3 -u bench.py > $O/bench.json 2> $O/bench.err &&
ARTIS_GPU_STATS=1 ARTIS_GPU_SO=artis_amd/lib/libartis_gpu_diag.so timeout -k 10 200 python3 -u bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/stamps.json 2> $O/stamps.err &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -u bench.py --no-cpu-baseline > $O/bench_prof.json 2> $O/bench_prof.err &&
B="python3 bench.py --packets 10000000 --steps 1 --warmup 0 --no-cpu-baseline" &&
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc/fetch -o run -- $B > $O/pmc/f.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmc/write -o run -- $B > $O/pmc/w.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc/lr -o run -- ./tools/linerate 32 400 > $O/pmc/lr.log 2>&1 &&
timeout -k 10 400 python3 -u bench.py --nts 30 --vpkt 4 --steps 1 --warmup 1 --no-cpu-baseline > $O/vpkt10m.json 2> $O/vpkt10m.err &&
timeout -k 10 600 python3 -u bench.py --packets 125000000 --steps 1 --warmup 0 --no-cpu-baseline > $O/big.json 2> $O/big.err
