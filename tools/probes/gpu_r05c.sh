# round 5: MSDA geometry-shared kernels -- parity, microbench A/B, step-graph tests
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_msda_gpu.py -q --timeout 200 --timeout-method thread > gpurun_out/c_msda_tests.log 2>&1 &&
timeout -k 10 300 python3 tools/msda_microbench.py --fwd-gs > gpurun_out/c_fwd_gs.jsonl 2>&1 &&
timeout -k 10 300 python3 tools/msda_microbench.py --bwd-variants --variant "sorted,sorted per-lane-geometry" > gpurun_out/c_bwd_gs.jsonl 2>&1 &&
timeout -k 10 900 python3 -u -m pytest tests/test_stepgraph_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/c_sg.log 2>&1 &&
timeout -k 10 600 python3 bench.py --no-cpu-baseline > gpurun_out/c_bench.log 2>&1
