#!/bin/bash
# A/B of the engine's launch knobs on the bench (1 timed step each): REFILL (k_rpkt idle lanes before a refill),
# REFILL_MA, MA_XCD (per-XCD queue ranges), MA_WAVES.
cd /root/repo
mkdir -p gpurun_out/knobs
B="python3 -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-update-grid"
i=0
for e in ARTIS_GPU_NONE=0 ARTIS_GPU_REFILL=16 ARTIS_GPU_REFILL=48 ARTIS_GPU_REFILL_MA=4 ARTIS_GPU_MA_XCD=1 ARTIS_GPU_MA_WAVES=5; do
  env $e timeout -k 10 200 $B > gpurun_out/knobs/b$i.json 2> gpurun_out/knobs/b$i.err || exit 1
  echo "$e" > gpurun_out/knobs/b$i.env
  i=$((i+1))
done
