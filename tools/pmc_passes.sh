cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
B="python3 bench.py --packets 1000000 --steps 1 --warmup 0 --no-cpu-baseline"
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc/fetch -o run -- $B > gpurun_out/pmc/f.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc/write -o run -- $B > gpurun_out/pmc/w.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -d gpurun_out/pmc/tcc -o run -- $B > gpurun_out/pmc/t.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_VALU SQ_WAVES --kernel-trace -d gpurun_out/pmc/sq -o run -- $B > gpurun_out/pmc/s.log 2>&1
