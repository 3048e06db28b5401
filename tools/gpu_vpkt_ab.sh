#!/bin/bash
# Virtual-packet line-walk prefetch depth A/B (ARTIS_VPKT_PF): parity tests per depth, then the vpkt bench.
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
for pf in 4 8 16; do
  ARTIS_VPKT_PF=$pf timeout -k 10 300 python -u -m pytest tests/test_gpu_vpkt.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_vpkt_tests_pf$pf.log 2>&1 || exit 1
  ARTIS_VPKT_PF=$pf timeout -k 10 300 python -u bench.py --nts 30 --vpkt 4 --packets 1000000 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/vpkt1m_pf$pf.json 2> gpurun_out/vpkt1m_pf$pf.err || exit 1
done
timeout -k 10 400 python -u bench.py --nts 30 --vpkt 4 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/vpkt10m.json 2> gpurun_out/vpkt10m.err
