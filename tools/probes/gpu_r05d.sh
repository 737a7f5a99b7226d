# round 5: step-graph GPU tests + the bench (protocol, ckpt-on line)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/test_stepgraph_gpu.py -v --timeout 300 --timeout-method thread > gpurun_out/d_sg.log 2>&1 ;
timeout -k 10 600 python3 bench.py --no-cpu-baseline > gpurun_out/d_bench.log 2>&1
