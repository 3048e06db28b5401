#!/bin/bash
# final measurement set, part A (RUN_TAG): GPU parity suite, rocprofv3 kernel statistics of the bench, FETCH_SIZE /
# WRITE_SIZE passes of the bench (separate runs) -> pmc summary keyed by the engine source hash, copied into this
# box's profiles/ so that the closing default bench line carries roofline.traffic
cd /root/repo
export TMPDIR=/tmp
T=${RUN_TAG:-r3w}
O=gpurun_out/$T
mkdir -p $O/pmc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 &&
tail -1 $O/gpu_tests.log &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -u bench.py --no-cpu-baseline --no-extra > $O/bench_prof.json 2> $O/bench_prof.err &&
B="python3 bench.py --packets 10000000 --steps 1 --warmup 0 --no-cpu-baseline --no-update-grid --no-extra" &&
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc/fetch -o run -- $B > $O/pmc/f.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmc/write -o run -- $B > $O/pmc/w.log 2>&1 &&
python3 tools/pmc_summary.py --fetch $O/pmc/fetch --write $O/pmc/write --packets 10000000 --ngrid 50 --nts 10 \
  --out $O/pmc_bench.json &&
cp $O/pmc_bench.json profiles/pmc_${T}_bench.json &&
timeout -k 10 500 python3 -u bench.py > $O/bench.json 2> $O/bench.err &&
tail -c 300 $O/bench.json
