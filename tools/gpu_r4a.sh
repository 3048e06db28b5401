cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r4a
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 &&
tail -1 $O/gpu_tests.log &&
timeout -k 10 500 python3 -u bench.py > $O/bench.json 2> $O/bench.err &&
tail -c 400 $O/bench.json
