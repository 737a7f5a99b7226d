# kernel-level breakdown of the sorted MSDA backward (rocprofv3 kernel trace)
set -o pipefail
mkdir -p gpurun_out/d_prof
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pd -o run -- python3 -u tools/msda_microbench.py --bwd-variants --iters 10 > gpurun_out/d_micro.log 2>&1
rc=$?
find /tmp/pd -name '*kernel_stats.csv' -exec cp {} gpurun_out/d_prof/ \;
python3 - <<'PY'
import csv, glob
for f in glob.glob("gpurun_out/d_prof/*kernel_stats.csv"):
    rows = list(csv.DictReader(open(f)))
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:25]:
        print(f'{float(r["AverageNs"])/1e3:10.1f} us avg {int(r["Calls"]):6d} calls  {r["Name"][:110]}')
PY
exit $rc
