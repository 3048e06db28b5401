#!/bin/bash
# A/B timing of engine builds (build/ab/<name>/libartis_gpu.so, tools/build_variants.sh; "main" = the in-tree
# artis_amd/lib/libartis_gpu.so) on the bench workload: tools/gpu_ab_so.sh name1[:ENV=V ...] name2 ...
# ENVS="X=1 Y=2" applies to every run; P packets (default 1e7).
cd /root/repo
mkdir -p gpurun_out
P=${P:-10000000}
for v in "$@"; do
  name=${v%%:*}; envs=""; [[ "$v" == *:* ]] && envs=${v#*:}
  so=build/ab/$name/libartis_gpu.so; [ "$name" = main ] && so=artis_amd/lib/libartis_gpu.so
  tag=$(echo "$v" | tr -c 'A-Za-z0-9_\n' '_')
  env ARTIS_GPU_SO=$so $ENVS $envs timeout -k 10 300 python3 bench.py --packets $P --steps 1 --warmup 1 \
    --no-cpu-baseline --no-update-grid --no-extra $BENCH_ARGS > gpurun_out/ab_$tag.json 2> gpurun_out/ab_$tag.err ||
    { echo "FAIL $v"; tail -5 gpurun_out/ab_$tag.err; exit 1; }
  grep "^\[artis_gpu\]" gpurun_out/ab_$tag.err | grep -v "^\[artis_gpu\] ma action [1-3578]" | sed "s/^/  $tag /"
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_'+sys.argv[1]+'.json').read().strip().splitlines()[-1]); print(sys.argv[2], 'value', round(d['value']), 'ms', round(d['ms_per_step']), 'precompute', round(d.get('precompute_ms', 0)), {k: round(x) for k, x in d['kernel_ms'].items()}, 'frac', round(d['roofline']['frac'], 4))" "$tag" "$v"
done
