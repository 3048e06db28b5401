#!/bin/bash
# round 3g: parity with the binned R queue and sorted spawns, then A/B of both
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_vpkt.py -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r3g_tests.log 2>&1 || { tail -40 gpurun_out/r3g_tests.log; exit 1; }
tail -3 gpurun_out/r3g_tests.log
B="--no-cpu-baseline --no-update-grid --no-extra --steps 2 --warmup 1"
timeout -k 10 300 python -u bench.py $B > gpurun_out/r3g_rbin1.json 2> gpurun_out/r3g_rbin1.err || exit 1
ARTIS_GPU_R_BIN=0 timeout -k 10 300 python -u bench.py $B > gpurun_out/r3g_rbin0.json 2> gpurun_out/r3g_rbin0.err || exit 1
V="--no-cpu-baseline --vpkt 4 --nts 30 --steps 1 --warmup 1"
timeout -k 10 400 python -u bench.py $V > gpurun_out/r3g_vsort1.json 2> gpurun_out/r3g_vsort1.err || exit 1
ARTIS_VPKT_SORT=0 timeout -k 10 400 python -u bench.py $V > gpurun_out/r3g_vsort0.json 2> gpurun_out/r3g_vsort0.err || exit 1
python - <<'PY'
import json
for f in ("rbin1", "rbin0", "vsort1", "vsort0"):
    d = json.loads(open(f"gpurun_out/r3g_{f}.json").read().strip().splitlines()[-1])
    print(f, round(d["value"]), round(d["ms_per_step"]), {k: round(v) for k, v in d["kernel_ms"].items()}, round(d["roofline"]["frac"], 4))
PY
