# kernel-trace stats of the instrumented step, eager vs HIP-graph replay
set -o pipefail
mkdir -p gpurun_out/b_eager gpurun_out/b_graph
export TMPDIR=/tmp
T() { timeout -k 10 "$@"; }
T 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pe -o run -- python3 -u tools/step_phases.py --steps 4 --warmup 2 > gpurun_out/b_eager.log 2>&1 &&
T 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pg -o run -- python3 -u tools/step_phases.py --steps 4 --warmup 2 --graphs > gpurun_out/b_graph.log 2>&1
rc=$?
find /tmp/pe -name '*kernel_stats.csv' -exec cp {} gpurun_out/b_eager/ \;
find /tmp/pg -name '*kernel_stats.csv' -exec cp {} gpurun_out/b_graph/ \;
for d in pe pg; do f=$(find /tmp/$d -name '*kernel_trace.csv' | head -n 1); [ -n "$f" ] && gzip -c "$f" > gpurun_out/b_${d}_trace.csv.gz; done
grep "{" gpurun_out/b_eager.log gpurun_out/b_graph.log
exit $rc
