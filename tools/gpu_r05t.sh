# round 5: the FFN's ReLU backward folded into the second Linear's dX kernel,
# the encoder query = src + pos with bf16 twins -- GPU suite, smoke, bench,
# kernel trace of the step graph
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/t_smoke.log 2>&1 || exit 1
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 8 --no-cpu-baseline --ckpt-compare off > gpurun_out/t_bench.json 2> gpurun_out/t_bench.err || exit 1
KEEP_TRACE=1 bash tools/gpu_session.sh census > gpurun_out/t_census.log 2>&1
