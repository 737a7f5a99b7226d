# round 5: GPU suite after the frozen-BERT path / cached masks / query-anchor
# kernel, then the bench line and a kernel census with the trace kept
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1200 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/j_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
case $rc in 134|139|124|137) exit 1;; esac
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 8 --no-cpu-baseline > gpurun_out/j_bench.json 2> gpurun_out/j_bench.err || exit 1
KEEP_TRACE=1 bash tools/gpu_session.sh census
