#!/usr/bin/env bash
# session-1 check: GPU parity tests, MSDA microbench A/B (tiled vs lane32), default bench
set -uo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -ra --timeout 300 --timeout-method thread \
    > gpurun_out/t1_gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
# a fault / abort / timeout ends the session here
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 300 python3 tools/msda_microbench.py > gpurun_out/t1_micro.log 2>&1 || exit $?
GD_MSDA_BWD=lane32 timeout -k 10 300 python3 tools/msda_microbench.py > gpurun_out/t1_micro_lane32.log 2>&1 || exit $?
timeout -k 10 600 python3 bench.py > gpurun_out/t1_bench.log 2>&1 || exit $?
exit $rc
