#!/bin/bash
# round 3i: restructured r-packet step + k_ma refill shifts: parity, then the bench A/B point
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r3i_tests.log 2>&1 || { tail -40 gpurun_out/r3i_tests.log; exit 1; }
tail -3 gpurun_out/r3i_tests.log
B="--no-cpu-baseline --no-update-grid --no-extra --steps 2 --warmup 1"
timeout -k 10 300 python -u bench.py $B > gpurun_out/r3i_bench.json 2> gpurun_out/r3i_bench.err || exit 1
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r3i_bench.json").read().strip().splitlines()[-1])
print("r3i", round(d["value"]), round(d["ms_per_step"]), {k: round(v) for k, v in d["kernel_ms"].items()}, round(d["roofline"]["frac"], 4))
PY
