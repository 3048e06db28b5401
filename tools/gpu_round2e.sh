#!/bin/bash
# Round-2e at the final engine sources: the full GPU parity suite, the bench line (incl. the update_grid solve),
# rocprofv3 kernel statistics of the bench, and the FETCH_SIZE / WRITE_SIZE passes of the bench configuration
# (separate rocprofv3 runs) that key roofline.traffic to this engine source hash.
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${RUN_TAG:-r2e}
mkdir -p $O/pmc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -u bench.py --no-cpu-baseline > $O/bench_prof.json 2> $O/bench_prof.err &&
B="python3 bench.py --packets 10000000 --steps 1 --warmup 0 --no-cpu-baseline --no-update-grid" &&
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc/fetch -o run -- $B > $O/pmc/f.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmc/write -o run -- $B > $O/pmc/w.log 2>&1
