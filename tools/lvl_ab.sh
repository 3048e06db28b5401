set -o pipefail
O=gpurun_out/r6y; mkdir -p $O
T=r6y bash tools/gpu.sh tests tests/test_gpu_parity.py || exit 1
for v in main old main old; do
  so=artis_amd/lib/libartis_gpu.so; [ $v = old ] && so=build/ab/old/libartis_gpu.so
  ARTIS_GPU_SO=$so timeout -k 10 300 python3 -u bench.py --baseline-config level_mode --steps 1 --warmup 1 --no-cpu-baseline > $O/lvl_$v.json 2> $O/lvl_$v.err || { echo FAIL $v; tail -5 $O/lvl_$v.err; exit 1; }
  python3 -c "
import json,sys
d=json.loads(open('$O/lvl_$v.json').read().strip().splitlines()[-1])
c=d.get('baseline_configs',d).get('level_mode_5x_lines') or d.get('level_mode_5x_lines')
print('$v', round(c['ms_per_step']), 'pre', round(c['precompute_ms']), {k: round(x) for k,x in c['kernel_ms'].items()})"
done
