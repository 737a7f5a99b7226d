set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/msda_microbench.py --enc-caps > gpurun_out/e_caps.log 2>&1 &&
timeout -k 10 60 rocprofv3 -L > gpurun_out/e_counters.txt 2>&1
rc=$?
tail -20 gpurun_out/e_caps.log
exit $rc
