cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_gamma.py tests/test_gpu_parity.py tests/test_golden.py tests/test_host_driver.py tests/test_spectrum.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests2.log 2>&1
