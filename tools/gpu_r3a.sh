#!/bin/bash
# Round 3, first call: the GPU parity suite at the current sources, the bench line, and the per-cell-table
# fallbacks timed at bench size: no line-coefficient table (gather walk), no macro-atom key
# cache (k_ma<false>), both.
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${RUN_TAG:-r3a}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 &&
timeout -k 10 400 python3 -u bench.py > $O/bench.json 2> $O/bench.err &&
ARTIS_GPU_NO_LINECOEF=1 timeout -k 10 400 python3 -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-update-grid > $O/bench_nolinecoef.json 2> $O/bench_nolinecoef.err &&
ARTIS_GPU_NO_MACACHE=1 timeout -k 10 600 python3 -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-update-grid > $O/bench_nomacache.json 2> $O/bench_nomacache.err &&
ARTIS_GPU_NO_LINECOEF=1 ARTIS_GPU_NO_MACACHE=1 timeout -k 10 600 python3 -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-update-grid > $O/bench_notables.json 2> $O/bench_notables.err
