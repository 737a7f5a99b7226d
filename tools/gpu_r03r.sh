# round-3 checkpoint: full GPU suite, driver bench command, kernel trace + PMC passes
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T() { timeout -k 10 "$@"; }
step() { echo "[$(date +%T)] $*"; }
step tests
T 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r_gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r_gpu_tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_session.sh benchprof || exit $?
python3 -c "
import json
for l in open('gpurun_out/s_bench.log'):
    if l.startswith('{'):
        d=json.loads(l); print('bench', round(d['value'],2), 'img/s', round(d['ms_per_step'],1), 'ms', d['step_ms'], d['roofline'])
"
head -3 gpurun_out/s_prof/steady_state.txt
