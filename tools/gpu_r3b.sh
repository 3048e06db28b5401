#!/bin/bash
# round 3: the nebular update_grid on the GPU (tests/test_gpu_nebular_update_grid.py) + the TE solver tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v -s --timeout 400 --timeout-method thread \
  tests/test_gpu_nebular_update_grid.py tests/test_gpu_te_solver.py > gpurun_out/r3b_tests.log 2>&1
rc=$?
grep -E "max rel diff|gpu .* ms|PASS|FAIL|outside|Error" gpurun_out/r3b_tests.log | tail -40
exit $rc
