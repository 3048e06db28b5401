#!/bin/bash
# round 3k: k_ma A/B over engine builds (tools/build_variants.sh): Philox cost, draw placement, streaming fetch, phases
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 900 bash tools/gpu_ab_so.sh base cheaprng rngearly ntfetch "stamps:ARTIS_GPU_STATS=1" > gpurun_out/r3k_ab.txt 2>&1
rc=$?; cat gpurun_out/r3k_ab.txt; exit $rc
