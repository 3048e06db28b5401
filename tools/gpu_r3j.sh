#!/bin/bash
# round 3j: the measurement set at the current engine sources: GPU parity suite, rocprof kernel statistics of the
# bench, FETCH_SIZE / WRITE_SIZE passes of the bench and of the config-5 vpkt shape (separate rocprofv3 runs), then
# the plain bench line with the CPU baseline.
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${RUN_TAG:-r3m}
mkdir -p $O/pmc $O/vpmc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 &&
tail -3 $O/gpu_tests.log &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -u bench.py --no-cpu-baseline --no-extra > $O/bench_prof.json 2> $O/bench_prof.err &&
B="python3 bench.py --packets 10000000 --steps 1 --warmup 0 --no-cpu-baseline --no-update-grid --no-extra" &&
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc/fetch -o run -- $B > $O/pmc/f.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmc/write -o run -- $B > $O/pmc/w.log 2>&1 &&
python3 tools/pmc_summary.py --fetch $O/pmc/fetch --write $O/pmc/write --packets 10000000 --ngrid 50 --nts 10 \
  --out $O/pmc_bench.json &&
V="python3 bench.py --packets 10000000 --nts 30 --vpkt 4 --steps 1 --warmup 0 --no-cpu-baseline --no-update-grid --no-extra" &&
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/vpmc/fetch -o run -- $V > $O/vpmc/f.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/vpmc/write -o run -- $V > $O/vpmc/w.log 2>&1 &&
python3 tools/pmc_summary.py --fetch $O/vpmc/fetch --write $O/vpmc/write --packets 10000000 --ngrid 50 --nts 30 \
  --vpkt 4 --out $O/pmc_vpkt.json &&
timeout -k 10 500 python3 -u bench.py > $O/bench.json 2> $O/bench.err &&
tail -c 600 $O/bench.json
