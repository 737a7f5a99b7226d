# full GPU suite on the committed tree, per-site attribution of the eager step
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T() { timeout -k 10 "$@"; }
step() { echo "[$(date +%T)] $*"; }
step tests
T 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/o_gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/o_gpu_tests.log; [ $rc -ne 0 ] && exit $rc
step torch-prof
T 400 python3 tools/torch_prof.py --out gpurun_out/o_tprof > gpurun_out/o_tprof.log 2>&1 || exit $?
head -60 gpurun_out/o_tprof_by_site.txt
