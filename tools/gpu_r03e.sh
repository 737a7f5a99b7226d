# sorted MSDA backward: parity, microbench, kernel breakdown
set -o pipefail
mkdir -p gpurun_out/e_prof
export TMPDIR=/tmp
T() { timeout -k 10 "$@"; }
T 600 python3 -u -m pytest tests/test_msda_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/e_msda_tests.log 2>&1
rc=$?
tail -3 gpurun_out/e_msda_tests.log
[ $rc -ne 0 ] && exit $rc
T 300 python3 -u tools/msda_microbench.py --bwd-variants > gpurun_out/e_micro.log 2>&1 || exit $?
cat gpurun_out/e_micro.log | grep geom | cut -c1-200
T 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pe -o run -- python3 -u tools/msda_microbench.py --bwd-variants --iters 10 > gpurun_out/e_micro_prof.log 2>&1
rc=$?
find /tmp/pe -name '*kernel_stats.csv' -exec cp {} gpurun_out/e_prof/ \;
f=$(find /tmp/pe -name '*kernel_trace.csv' | head -n 1); [ -n "$f" ] && gzip -c "$f" > gpurun_out/e_prof/trace.csv.gz
exit $rc
