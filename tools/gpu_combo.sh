# encoder-backward probes, then the HIP-graph trial (risky step last)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/msda_microbench.py --enc-probes > gpurun_out/e_probes.log 2>&1 &&
bash tools/gpu_graphs.sh
rc=$?
tail -12 gpurun_out/e_probes.log | cut -c1-200
exit $rc
