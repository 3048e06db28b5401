#!/bin/bash
# Occupancy A/B for the two FP64-heavy persistent kernels: k_vpkt (ARTIS_VPKT_OCC 1/2/3) and k_rpkt
# (ARTIS_GPU_RPKT_OCC 1/2); parity tests under each variant, then the bench.
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
for o in 2 3 1; do
  ARTIS_VPKT_OCC=$o timeout -k 10 300 python -u -m pytest tests/test_gpu_vpkt.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_vpkt_tests_occ$o.log 2>&1 || exit 1
  ARTIS_VPKT_OCC=$o timeout -k 10 300 python -u bench.py --nts 30 --vpkt 4 --packets 1000000 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/vpkt1m_occ$o.json 2> gpurun_out/vpkt1m_occ$o.err || exit 1
done
ARTIS_GPU_RPKT_OCC=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_parity_rocc2.log 2>&1 || exit 1
for o in 2 1; do
  ARTIS_GPU_RPKT_OCC=$o timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_rocc$o.json 2> gpurun_out/bench_rocc$o.err || exit 1
done
