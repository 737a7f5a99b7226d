# round 5 (session 2): count kernel with 4 rounds per workgroup, wave-scan
# prefix sums -- MSDA GPU tests, then a kernel trace of the sorted backward
# at the encoder shape (init geometry and 2-px spread)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_msda_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/w_msda_tests.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/w_prof -o run -- python3 tools/msda_microbench.py --bwd-variants --variant "sorted,sorted count-r1,lane32" --iters 20 > gpurun_out/w_mb.log 2>&1 || exit 1
find /tmp/w_prof -name '*kernel_stats.csv' -exec cp {} gpurun_out/w_kernel_stats.csv \;
