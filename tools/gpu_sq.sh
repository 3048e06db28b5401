#!/bin/bash
# SQ instruction counters of the bench kernels (one rocprofv3 --pmc pass) + optional bench A/B via ENVS.
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/sq
rm -rf gpurun_out/sq/db
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM --kernel-trace -d gpurun_out/sq/db -o run -- python3 bench.py --packets ${P:-2000000} --steps 1 --warmup 0 --no-cpu-baseline --no-update-grid --no-extra > gpurun_out/sq/sq.log 2>&1 || exit 1
i=0
for e in ${ENVS}; do
  env $e ARTIS_GPU_STATS=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/sq/bench$i.json 2> gpurun_out/sq/bench$i.err || exit 1
  echo "$e" >> gpurun_out/sq/bench$i.err
  i=$((i+1))
done
