#!/bin/bash
# round 3: the nebular update_grid on the GPU (tests/test_gpu_nebular_update_grid.py), the TE solver tests, and a
# kernel-time profile of one one-zone solve
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v -s --timeout 400 --timeout-method thread \
  tests/test_gpu_nebular_update_grid.py tests/test_gpu_te_solver.py > gpurun_out/r3b_tests.log 2>&1
rc=$?
grep -E "max diff|max rel diff|gpu .* ms|element|PASS|FAIL|outside|Error" gpurun_out/r3b_tests.log | tail -50
if [ $rc -ne 0 ] && grep -q -E "illegal memory|APERTURE|Memory access fault" gpurun_out/r3b_tests.log; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3b_prof -o nl -- python3 tools/nl_prof.py onezone > gpurun_out/r3b_prof.log 2>&1 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3b_profm -o nl -- python3 tools/nl_prof.py multi > gpurun_out/r3b_profm.log 2>&1
prc=$?
tail -3 gpurun_out/r3b_prof.log
exit $(( rc != 0 ? rc : prc ))
