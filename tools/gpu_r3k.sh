#!/bin/bash
# round 3k: gamma GPU parity (incl. the Compton emissivity estimators), then k_ma A/B over engine builds
# (tools/build_variants.sh): Philox cost, draw placement, streaming fetch, meta load without a dead word, phases
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_gamma.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/r3k_gamma.log 2>&1
rc=$?; tail -4 gpurun_out/r3k_gamma.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 bash tools/gpu_ab_so.sh base meta3 cheaprng rngearly ntfetch "stamps:ARTIS_GPU_STATS=1" > gpurun_out/r3k_ab.txt 2>&1
rc=$?; cat gpurun_out/r3k_ab.txt; exit $rc
