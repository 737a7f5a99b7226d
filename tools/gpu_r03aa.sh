# K1 with level-loaded locations (146 VGPRs, 3 waves/SIMD): parity, microbench, per-geometry breakdown
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T() { timeout -k 10 "$@"; }
step() { echo "[$(date +%T)] $*"; }
step parity
T 600 python3 -u -m pytest tests/test_msda_gpu.py -x -q --timeout 120 --timeout-method thread -k "sorted or init_geometry" > gpurun_out/aa_parity.log 2>&1
rc=$?; tail -2 gpurun_out/aa_parity.log; [ $rc -ne 0 ] && exit $rc
step microbench
for v in "sorted" "sorted level-loaded"; do
  for g in enc-init enc-spread2; do
    T 120 python3 tools/msda_microbench.py --bwd-variants --iters 50 --geom $g --variant "$v" >> gpurun_out/aa_bwd_variants.jsonl 2>&1 || exit $?
  done
done
grep -v amdgpu.ids gpurun_out/aa_bwd_variants.jsonl | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['geom'], d['variant'], round(d['bwd_us'], 1))
"
R=$GRAFT_REPO_ROOT
for geom in enc-init enc-spread2; do
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/aa_$geom -o run -- python3 $R/tools/msda_microbench.py --bwd-variants --geom $geom --variant "sorted level-loaded" --iters 10 > $R/gpurun_out/aa_$geom.log 2>&1 || exit $?
  cd $R
  f=$(find /tmp/aa_$geom -name '*kernel_stats.csv' | head -n 1)
  cp "$f" gpurun_out/aa_${geom}_kernel_stats.csv
  echo "== $geom"
  python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if any(k in r['Name'] for k in ('msda_bwd', 'scan_')):
        print(round(float(r['AverageNs'])/1e3, 1), 'us avg', r['Calls'], r['Name'][:100])
"
done
