# token-major BiAttention, HIP LayerNorm for Swin, sweep rows <= 8 + offset prefetch:
# parity (kernels, blocks, full size), microbench, bench, per-site attribution
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T() { timeout -k 10 "$@"; }
step() { echo "[$(date +%T)] $*"; }
step parity
T 900 python3 -u -m pytest tests/test_kernels_gpu.py tests/test_msda_gpu.py tests/test_blocks_gpu.py tests/test_fullsize_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/p_parity.log 2>&1
rc=$?; tail -2 gpurun_out/p_parity.log; [ $rc -ne 0 ] && exit $rc
step microbench
T 300 python3 tools/msda_microbench.py --bwd-variants --iters 20 > gpurun_out/p_bwd_variants.jsonl 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/p_bwd_variants.jsonl | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['geom'], d['variant'], round(d['bwd_us'], 1))
"
step bench
T 400 python3 bench.py --no-cpu-baseline > gpurun_out/p_bench.log 2>&1 || exit $?
python3 -c "
import json
for l in open('gpurun_out/p_bench.log'):
    if l.startswith('{'):
        d=json.loads(l); print('bench', round(d['value'],2), 'img/s', round(d['ms_per_step'],1), 'ms', d['roofline']['avg_launch_us'], d['loss'])
"
step torch-prof
T 400 python3 tools/torch_prof.py --out gpurun_out/p_tprof > gpurun_out/p_tprof.log 2>&1
head -40 gpurun_out/p_tprof_by_site.txt
