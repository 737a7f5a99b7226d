set -o pipefail
mkdir -p gpurun_out/g_prof
export TMPDIR=/tmp
T() { timeout -k 10 "$@"; }
T 600 python3 -u -m pytest tests/test_msda_gpu.py -x -q --timeout 120 --timeout-method thread -k "sorted or pixel_block or init_geometry or gradcheck or golden" > gpurun_out/g_msda_tests.log 2>&1
rc=$?
tail -3 gpurun_out/g_msda_tests.log
[ $rc -ne 0 ] && exit $rc
T 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pg -o run -- python3 -u tools/msda_microbench.py --bwd-variants --iters 5 > gpurun_out/g_micro_prof.log 2>&1
rc=$?
grep geom gpurun_out/g_micro_prof.log | cut -c1-110
f=$(find /tmp/pg -name '*kernel_trace.csv' | head -n 1); [ -n "$f" ] && gzip -c "$f" > gpurun_out/g_prof/trace.csv.gz
exit $rc
