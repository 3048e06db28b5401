#!/bin/bash
# Random-line fetch rate (tools/linerate) + SQ counters of the bench's kernels at 1e6 packets.
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/lr
timeout -k 10 180 ./tools/linerate 32 400 > gpurun_out/lr/linerate.txt 2>&1

