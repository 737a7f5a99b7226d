# round-3 checkpoint after re-entry: driver bench command, full GPU suite, rocprof stats of the bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T() { timeout -k 10 "$@"; }
step() { echo "[$(date +%T)] $*"; }
step bench
T 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/l_bench.log 2>&1 || exit $?
python3 -c "
import json
for l in open('gpurun_out/l_bench.log'):
    if l.startswith('{'):
        d=json.loads(l); print('bench', round(d['value'],2), 'img/s', round(d['ms_per_step'],1), 'ms', d.get('step_ms'), d['roofline'])
"
step tests
T 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/l_gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/l_gpu_tests.log
[ $rc -ne 0 ] && exit $rc
step rocprof
T 500 rocprofv3 --kernel-trace --stats -d gpurun_out/l_prof -o run -- python3 bench.py --steps 10 --warmup 5 --no-cpu-baseline > gpurun_out/l_prof.log 2>&1
