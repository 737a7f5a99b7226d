# round 5: the step-graph GPU tests (capture-once, cache stream, forced
# failure fallback, 1-rank RCCL capture), then the bench with the new protocol
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/test_stepgraph_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/b_sg.log 2>&1 &&
timeout -k 10 600 python3 bench.py --no-cpu-baseline > gpurun_out/b_bench.log 2>&1
