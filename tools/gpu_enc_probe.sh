# encoder-backward phase probes (tools/msda_microbench.py --enc-probes)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/msda_microbench.py --enc-probes > gpurun_out/e_probes.log 2>&1
rc=$?
tail -20 gpurun_out/e_probes.log
exit $rc
