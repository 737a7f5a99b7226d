# MSDA microbench (decoder backward A/B vs r02b), encoder-backward probes,
# MSDA parity tests, then the HIP-graph trial (the risky step last)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/msda_microbench.py > gpurun_out/e_micro.log 2>&1 &&
timeout -k 10 300 python3 tools/msda_microbench.py --enc-probes > gpurun_out/e_probes.log 2>&1 &&
timeout -k 10 300 python3 -u -m pytest tests/test_msda_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/e_msda_tests.log 2>&1 &&
bash tools/gpu_graphs.sh
rc=$?
tail -4 gpurun_out/e_micro.log | cut -c1-300
tail -12 gpurun_out/e_probes.log | cut -c1-200
tail -2 gpurun_out/e_msda_tests.log
exit $rc
