#!/bin/bash
# round 3h: per-pass wave diagnostics compiled out; k_rpkt occupancy 1 vs 2
set -o pipefail
mkdir -p gpurun_out
B="--no-cpu-baseline --no-update-grid --no-extra --steps 2 --warmup 1"
timeout -k 10 300 python -u bench.py $B > gpurun_out/r3h_nostats.json 2> gpurun_out/r3h_nostats.err || exit 1
ARTIS_GPU_RPKT_OCC=1 timeout -k 10 300 python -u bench.py $B > gpurun_out/r3h_occ1.json 2> gpurun_out/r3h_occ1.err || exit 1
python - <<'PY'
import json
for f in ("nostats", "occ1"):
    d = json.loads(open(f"gpurun_out/r3h_{f}.json").read().strip().splitlines()[-1])
    print(f, round(d["value"]), round(d["ms_per_step"]), {k: round(v) for k, v in d["kernel_ms"].items()}, round(d["roofline"]["frac"], 4))
PY
