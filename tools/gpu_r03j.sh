# round-3 checkpoint: full GPU test suite, default bench (graphs) + eager A/B + forward-only
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/fullsize_margins.jsonl
T() { timeout -k 10 "$@"; }
step() { echo "[$(date +%T)] $*"; }
step tests
T 1100 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/j_gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/j_gpu_tests.log
[ $rc -ne 0 ] && exit $rc
step bench
T 400 python3 bench.py > gpurun_out/j_bench.log 2>&1 || exit $?
step bench-eager
T 400 python3 bench.py --no-graphs --no-cpu-baseline > gpurun_out/j_bench_eager.log 2>&1 || exit $?
step bench-fwd
T 400 python3 bench.py --forward-only --no-cpu-baseline > gpurun_out/j_bench_fwd.log 2>&1 || exit $?
for f in j_bench j_bench_eager j_bench_fwd; do python3 -c "
import json
for l in open('gpurun_out/$f.log'):
    if l.startswith('{'):
        d=json.loads(l); print('$f', round(d['value'],2), 'img/s', round(d['ms_per_step'],1), 'ms', d.get('step_ms'), d['roofline'] and round(d['roofline']['avg_launch_us'],1), d['options'].get('hip_graphs'))
"; done
