set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "window or swin or fullsize or blocks" > gpurun_out/w_tests.log 2>&1 &&
timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/w_bench.log 2>&1 &&
GD_WATTN_REGSUM=0 timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/w_bench_noreg.log 2>&1
rc=$?
tail -5 gpurun_out/w_tests.log
exit $rc
