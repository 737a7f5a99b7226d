# sorted MSDA backward v2 (count pass + direct record writes) and attention
# wave tilings: parity, microbench, bench, kernel trace
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T() { timeout -k 10 "$@"; }
step() { echo "[$(date +%T)] $*"; }
step parity
T 600 python3 -u -m pytest tests/test_msda_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/m_parity.log 2>&1
rc=$?; tail -2 gpurun_out/m_parity.log; [ $rc -ne 0 ] && exit $rc
step microbench
T 300 python3 tools/msda_microbench.py --bwd-variants --iters 20 > gpurun_out/m_bwd_variants.jsonl 2>&1 || exit $?
step bench
T 400 python3 bench.py --no-cpu-baseline > gpurun_out/m_bench.log 2>&1 || exit $?
python3 -c "
import json
for l in open('gpurun_out/m_bench.log'):
    if l.startswith('{'):
        d=json.loads(l); print('bench', round(d['value'],2), 'img/s', round(d['ms_per_step'],1), 'ms', d['roofline']['avg_launch_us'])
        for k,v in d['hip_entry_points_one_step'].items(): print(k, v)
"
step trace
T 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/m_prof -o run -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 2 > gpurun_out/m_prof.log 2>&1 || exit $?
mkdir -p gpurun_out/m_prof
find /tmp/m_prof -name '*stats*.csv' -exec cp {} gpurun_out/m_prof/ \;
kt=$(find /tmp/m_prof -name '*kernel_trace.csv' | head -n 1)
python3 tools/trace_steps.py --skip 2 "$kt" > gpurun_out/m_prof/steady_state.txt 2>&1
head -3 gpurun_out/m_prof/steady_state.txt
