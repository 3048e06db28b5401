# level-mode A/B (bench.py --baseline-config level_mode, one warm + one timed step) over engine builds:
#   bash tools/lvl_ab.sh name[:ENV=V] ...   (name main = the in-tree library, otherwise build/ab/<name>)
set -o pipefail
O=gpurun_out/${T:-r6y}; mkdir -p $O
for v in "$@"; do
  name=${v%%:*}; envs=""; [[ "$v" == *:* ]] && envs=${v#*:}
  so=artis_amd/lib/libartis_gpu.so; [ "$name" != main ] && so=build/ab/$name/libartis_gpu.so
  tag=$(echo "$v" | tr -c 'A-Za-z0-9_\n' '_')
  env ARTIS_GPU_SO=$so $envs timeout -k 10 300 python3 -u bench.py --baseline-config level_mode --steps 1 --warmup 1 \
    --no-cpu-baseline > $O/lvl_$tag.json 2> $O/lvl_$tag.err || { echo FAIL $v; tail -5 $O/lvl_$tag.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/lvl_$tag.json').read().strip().splitlines()[-1])
c=d.get('baseline_configs',d).get('level_mode_5x_lines') or d.get('level_mode_5x_lines')
print('$v', round(c['ms_per_step']), 'pre', round(c['precompute_ms']), {k: round(x) for k,x in c['kernel_ms'].items()})"
done
