#!/bin/bash
# The 5x-lines atom (470 745 lines, --line-window 160) on the 50^3 grid: level-mode macro-atom records.
# Usage: tools/gpu_x5.sh PACKETS STEPS [ENV=V ...]   (each run under its own time limit LIMIT, default 500 s;
# BENCH_EXTRA: more bench.py arguments, e.g. "--ngrid 30")
cd /root/repo || exit 1
export TMPDIR=/tmp
O=${O:-gpurun_out/x5}
mkdir -p "$O"
P=$1; S=$2; shift 2
tag=$(echo "p$P $BENCH_EXTRA $*" | tr -c 'A-Za-z0-9_\n' '_')
env "$@" timeout -k 10 ${LIMIT:-500} python3 -u bench.py --line-window 160 --max-lines 1000000 --packets "$P" --steps "$S" \
  --warmup 1 --no-cpu-baseline --no-update-grid --no-extra $BENCH_EXTRA > "$O/$tag.json" 2> "$O/$tag.err"
rc=$?
grep -v amdgpu.ids "$O/$tag.err" | grep -v running | tail -6
[ $rc -eq 0 ] && python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'ms', round(d['ms_per_step']), 'ma', round(d['kernel_ms']['ma']), 'ps/jump', round(d['ma_ps_per_jump'], 1), 'rounds', d['event_rounds'], 'tables', {k: d['tables'][k] for k in ('ma_jumps_recorded', 'ma_jumps', 'ma_level_records')})" "$O/$tag.json" "$tag"
exit $rc
