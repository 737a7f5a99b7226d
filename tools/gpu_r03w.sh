# sweep record prefetch A/B, per-kernel breakdown of the sorted backward
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T() { timeout -k 10 "$@"; }
step() { echo "[$(date +%T)] $*"; }
step parity
T 600 python3 -u -m pytest tests/test_msda_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/w_parity.log 2>&1
rc=$?; tail -2 gpurun_out/w_parity.log; [ $rc -ne 0 ] && exit $rc
step microbench
T 300 python3 tools/msda_microbench.py --bwd-variants --iters 20 > gpurun_out/w_bwd_variants.jsonl 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/w_bwd_variants.jsonl | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['geom'], d['variant'], round(d['bwd_us'], 1))
"
step trace
cd /tmp && T 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/w_prof -o run -- python3 $GRAFT_REPO_ROOT/tools/msda_microbench.py --bwd-variants --iters 5 > $GRAFT_REPO_ROOT/gpurun_out/w_prof.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/w_prof
find /tmp/w_prof -name '*kernel_stats.csv' -exec cp {} gpurun_out/w_prof/ \;
python3 -c "
import csv, glob
f = glob.glob('gpurun_out/w_prof/*kernel_stats.csv')[0]
for r in csv.DictReader(open(f)):
    if any(k in r['Name'] for k in ('msda_bwd', 'scan_')):
        print(round(float(r['AverageNs'])/1e3, 1), 'us avg', r['Calls'], r['Name'][:110])
"
