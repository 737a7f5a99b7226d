# round-3 checkpoint with the level-loaded per-sample pass: smoke, full GPU suite, the driver's bench command,
# kernel trace of the graph-mode bench, filtered PMC passes of the MSDA kernels
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T() { timeout -k 10 "$@"; }
step() { echo "[$(date +%T)] $*"; }
step smoke
T 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/ab_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/ab_smoke.log
step tests
T 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/ab_gpu_tests.log; [ $rc -ne 0 ] && exit $rc
step bench
T 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/ab_bench.log 2>&1 || exit $?
python3 -c "
import json
for l in open('gpurun_out/ab_bench.log'):
    if l.startswith('{'):
        d=json.loads(l); print('bench', round(d['value'],2), 'img/s', round(d['ms_per_step'],1), 'ms', d['step_ms'], d['roofline'])
"
step bench-no-shadows
GDINO_CAST_SHADOWS=0 T 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ab_bench_noshadow.log 2>&1 || exit $?
python3 -c "
import json
for l in open('gpurun_out/ab_bench_noshadow.log'):
    if l.startswith('{'):
        d=json.loads(l); print('bench no-shadows', round(d['value'],2), 'img/s', round(d['ms_per_step'],1), 'ms', d['step_ms'])
"
step trace
cd /tmp && T 500 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ab_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 3 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/ab_prof.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab_prof
find /tmp/ab_prof -name '*stats*.csv' -exec cp {} gpurun_out/ab_prof/ \;
kt=$(find /tmp/ab_prof -name '*kernel_trace.csv' | head -n 1)
python3 tools/trace_steps.py --skip 2 "$kt" > gpurun_out/ab_prof/steady_state.txt 2>&1
head -3 gpurun_out/ab_prof/steady_state.txt
bash tools/gpu_r03s.sh
