#!/bin/bash
# End of round 2: the measurement set of tools/gpu_round2e.sh at the final sources, plus the plain bench line with
# the CPU baseline.
cd /root/repo
RUN_TAG=r2g bash tools/gpu_round2e.sh &&
timeout -k 10 400 python3 -u bench.py > gpurun_out/r2g/bench.json 2> gpurun_out/r2g/bench.err
