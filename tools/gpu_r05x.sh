# round 5 (session 2): count kernel 4 rounds per workgroup, wave-scan prefix
# sums in 2 launches -- GPU suite, smoke, the sorted backward alone, the
# driver's bench command, its kernel trace and PMC traffic passes
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/x_gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/x_smoke.log 2>&1 || exit 1
timeout -k 10 300 python3 tools/msda_microbench.py --bwd-variants --variant "sorted,sorted count-r1,sorted count-r8" --iters 20 > gpurun_out/x_mb.log 2>&1 || exit 1
bash tools/gpu_session.sh benchprof > gpurun_out/x_benchprof.log 2>&1
