#!/bin/bash
# A/B timing of engine variants (env toggles) on the bench workload; one JSON summary line per variant
P=${P:-1000000}
for v in "$@"; do
  env $v timeout -k 10 300 python bench.py --packets $P --steps 1 --warmup 1 --no-cpu-baseline $BENCH_ARGS > gpurun_out/ab.json 2>gpurun_out/ab.err || { echo "FAIL $v"; tail -3 gpurun_out/ab.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1]); print(sys.argv[1], 'transport_ms', round(d['transport_ms'],1), 'precompute_ms', round(d['precompute_ms'],1), 'rounds', d['event_rounds'], 'value', round(d['value']), 'kernel_ms', {k: round(v,1) for k,v in d['kernel_ms'].items()}, 'ma_jumps/pkt', round(d['work_per_packet']['ma_jumps']))" "$v"
done
