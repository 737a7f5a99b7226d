# end-to-end: eager bench (sorted MSDA backward default) + graph-mode kernel trace vs eager
set -o pipefail
mkdir -p gpurun_out/h_eager gpurun_out/h_graph
export TMPDIR=/tmp
T() { timeout -k 10 "$@"; }
T 400 python3 bench.py --no-cpu-baseline > gpurun_out/h_bench.log 2>&1 || exit $?
python3 -c "
import json
for l in open('gpurun_out/h_bench.log'):
    if l.startswith('{'):
        d=json.loads(l); print('bench', round(d['value'],2), 'img/s', round(d['ms_per_step'],1), 'ms', d['step_ms'], d['roofline'])
"
T 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/he -o run -- python3 -u tools/step_phases.py --steps 3 --warmup 2 > gpurun_out/h_eager.log 2>&1 &&
T 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/hg -o run -- python3 -u tools/step_phases.py --steps 3 --warmup 2 --graphs > gpurun_out/h_graph.log 2>&1
rc=$?
for d in he hg; do f=$(find /tmp/$d -name '*kernel_trace.csv' | head -n 1); [ -n "$f" ] && gzip -c "$f" > gpurun_out/h_${d}_trace.csv.gz; done
grep "{" gpurun_out/h_eager.log gpurun_out/h_graph.log
exit $rc
