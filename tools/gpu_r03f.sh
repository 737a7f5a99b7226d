set -o pipefail
mkdir -p gpurun_out/f_prof
export TMPDIR=/tmp
T() { timeout -k 10 "$@"; }
T 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pf -o run -- python3 -u tools/msda_microbench.py --bwd-variants --iters 5 > gpurun_out/f_micro_prof.log 2>&1
rc=$?
grep geom gpurun_out/f_micro_prof.log | cut -c1-130
f=$(find /tmp/pf -name '*kernel_trace.csv' | head -n 1); [ -n "$f" ] && gzip -c "$f" > gpurun_out/f_prof/trace.csv.gz
exit $rc
