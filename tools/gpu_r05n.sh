# round 5: GPU suite, smoke (pinned loss), bench line, census with the trace
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1200 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/n_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
case $rc in 134|139|124|137) exit 1;; esac
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/n_smoke.log 2>&1 || exit 1
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 8 --no-cpu-baseline > gpurun_out/n_bench.json 2> gpurun_out/n_bench.err || exit 1
KEEP_TRACE=1 bash tools/gpu_session.sh census
