#!/bin/bash
# round 3p: what the driver runs at round end, on the final tree: smoke(), then the default bench line (which must
# pick up profiles/pmc_r03m_bench.json at the same engine hash)
cd /root/repo
mkdir -p gpurun_out/r3p
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3p/smoke.log 2>&1 &&
tail -2 gpurun_out/r3p/smoke.log &&
timeout -k 10 600 python3 -u bench.py > gpurun_out/r3p/bench.json 2> gpurun_out/r3p/bench.err
rc=$?; tail -c 800 gpurun_out/r3p/bench.json; exit $rc
