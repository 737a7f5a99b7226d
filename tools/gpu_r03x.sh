# per-kernel breakdown of the default sorted backward at each geometry
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for geom in enc-init enc-spread2; do
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/x_$geom -o run -- python3 $R/tools/msda_microbench.py --bwd-variants --geom $geom --variant sorted --iters 10 > $R/gpurun_out/x_$geom.log 2>&1 || exit $?
  cd $R
  f=$(find /tmp/x_$geom -name '*kernel_stats.csv' | head -n 1)
  cp "$f" gpurun_out/x_${geom}_kernel_stats.csv
  echo "== $geom"
  python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if any(k in r['Name'] for k in ('msda_bwd', 'scan_')):
        print(round(float(r['AverageNs'])/1e3, 1), 'us avg', r['Calls'], r['Name'][:100])
"
done
