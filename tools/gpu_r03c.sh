# sorted MSDA backward: parity tests, then microbench vs enc / lane32
set -o pipefail
mkdir -p gpurun_out
T() { timeout -k 10 "$@"; }
T 600 python3 -u -m pytest tests/test_msda_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/c_msda_tests.log 2>&1
rc=$?
tail -5 gpurun_out/c_msda_tests.log
[ $rc -ne 0 ] && exit $rc
T 300 python3 -u tools/msda_microbench.py --bwd-variants > gpurun_out/c_micro.log 2>&1
rc=$?
tail -20 gpurun_out/c_micro.log
exit $rc
