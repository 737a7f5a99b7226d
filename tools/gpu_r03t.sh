# level-by-level per-sample pass: parity, microbench, bench, then the filtered PMC passes
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T() { timeout -k 10 "$@"; }
step() { echo "[$(date +%T)] $*"; }
step parity
T 900 python3 -u -m pytest tests/test_msda_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_parity.log 2>&1
rc=$?; tail -2 gpurun_out/t_parity.log; [ $rc -ne 0 ] && exit $rc
step microbench
T 300 python3 tools/msda_microbench.py --bwd-variants --iters 20 > gpurun_out/t_bwd_variants.jsonl 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/t_bwd_variants.jsonl | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['geom'], d['variant'], round(d['bwd_us'], 1))
"
step bench
T 400 python3 bench.py --no-cpu-baseline > gpurun_out/t_bench.log 2>&1 || exit $?
python3 -c "
import json
for l in open('gpurun_out/t_bench.log'):
    if l.startswith('{'):
        d=json.loads(l); print('bench', round(d['value'],2), 'img/s', round(d['ms_per_step'],1), 'ms', d['roofline']['avg_launch_us'], d['loss'])
"
bash tools/gpu_r03s.sh
