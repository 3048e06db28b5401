#!/bin/bash
# final measurement set, part B (RUN_TAG): the config-5 shape (1e7 packets, timestep 30, 4 observers): FETCH_SIZE /
# WRITE_SIZE passes -> pmc summary (copied into this box's profiles/), then its bench line under rocprofv3 statistics
cd /root/repo
export TMPDIR=/tmp
T=${RUN_TAG:-r3w}
O=gpurun_out/$T
mkdir -p $O/vpmc
V="python3 bench.py --packets 10000000 --nts 30 --vpkt 4 --steps 1 --warmup 0 --no-cpu-baseline --no-update-grid --no-extra" &&
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/vpmc/fetch -o run -- $V > $O/vpmc/f.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/vpmc/write -o run -- $V > $O/vpmc/w.log 2>&1 &&
python3 tools/pmc_summary.py --fetch $O/vpmc/fetch --write $O/vpmc/write --packets 10000000 --ngrid 50 --nts 30 \
  --vpkt 4 --out $O/pmc_vpkt.json &&
cp $O/pmc_vpkt.json profiles/pmc_${T}_vpkt.json &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/vprof -o run -- python3 -u bench.py --packets 10000000 --nts 30 --vpkt 4 --steps 1 --warmup 1 --no-cpu-baseline --no-update-grid --no-extra > $O/bench_vpkt.json 2> $O/bench_vpkt.err &&
tail -c 300 $O/bench_vpkt.json
