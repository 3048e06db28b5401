#!/bin/bash
# Parity tests (GPU_TESTS, default the core parity file) then a short bench with wave statistics.
# ENVS: extra environment assignments for the bench A/B (e.g. "ARTIS_GPU_MA_WAVES=2"), one bench per entry.
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/q
[ "${GPU_TESTS}" = none ] || timeout -k 10 600 python -u -m pytest ${GPU_TESTS:-tests/test_gpu_parity.py} -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/q/tests.log 2>&1 || exit 1
i=0
for e in ${ENVS:-NONE=1}; do
  env $e ARTIS_GPU_STATS=1 timeout -k 10 300 python -u bench.py --steps ${STEPS:-2} --warmup 1 --no-cpu-baseline $BENCH_ARGS > gpurun_out/q/bench$i.json 2> gpurun_out/q/bench$i.err || exit 1
  echo "$e" >> gpurun_out/q/bench$i.err
  i=$((i+1))
done
