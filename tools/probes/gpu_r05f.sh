# round 5: step-graph GPU tests (capture-failure fallback, cache stream, text
# buckets), each test file under its own time limit
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/test_stepgraph_gpu.py -v --timeout 300 --timeout-method thread > gpurun_out/f_sg.log 2>&1
