# round 5: step-graph GPU tests after the watchdog / shadow-cache fixes, the
# attention kernel tests (device dropout seed), then a short bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/test_stepgraph_gpu.py -v --timeout 300 --timeout-method thread > gpurun_out/g_sg.log 2>&1
rc1=$?
timeout -k 10 600 python3 -u -m pytest tests/test_kernels_gpu.py -v -k "attn or attention" --timeout 120 --timeout-method thread > gpurun_out/g_attn.log 2>&1
rc2=$?
echo "rc stepgraph=$rc1 attn=$rc2"
case $rc1$rc2 in *134*|*139*|*124*|*137*) exit 1;; esac
timeout -k 10 600 python3 -u bench.py --steps 20 --warmup 8 > gpurun_out/g_bench.json 2> gpurun_out/g_bench.err
