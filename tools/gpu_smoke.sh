# round-end rehearsal: smoke() and the GPU suite on the final tree
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/z_smoke.log 2>&1 &&
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/z_tests.log 2>&1
rc=$?
tail -2 gpurun_out/z_smoke.log; tail -2 gpurun_out/z_tests.log
exit $rc
