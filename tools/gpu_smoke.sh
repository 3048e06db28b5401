#!/bin/bash
# smoke() on the final tree, as the driver runs it at round end
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1
rc=$?; tail -2 gpurun_out/smoke_final.log; exit $rc
