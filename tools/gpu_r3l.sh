#!/bin/bash
# round 3l: full GPU parity suite (radiative deactivation's line index looked up by ma_finish, Compton estimators),
# then k_ma A/B: deferred line index alone / + 3-word meta load / + paired draws, and the load-wait phase stamps
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3l_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3l_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 bash tools/gpu_ab_so.sh defer meta3 paired_meta3 "twait:ARTIS_GPU_STATS=1" > gpurun_out/r3l_ab.txt 2>&1
rc=$?; cat gpurun_out/r3l_ab.txt; exit $rc
