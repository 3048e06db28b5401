#!/bin/bash
# round 3: smoke() and the default bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3c_smoke.log 2>&1 || { tail -20 gpurun_out/r3c_smoke.log; exit 1; }
tail -2 gpurun_out/r3c_smoke.log
timeout -k 10 900 python -u bench.py > gpurun_out/r3c_bench.json 2> gpurun_out/r3c_bench.err
rc=$?
tail -3 gpurun_out/r3c_bench.err
exit $rc
