# graphs with the split-K / fp32-output weight gradients inside the capture
set -o pipefail
mkdir -p gpurun_out
T() { timeout -k 10 "$@"; }
T 420 python3 -u tools/graph_probe.py check 800 1333 > gpurun_out/i_check.log 2>&1 &&
T 300 python3 -u tools/step_phases.py --graphs > gpurun_out/i_phases_g.log 2>&1 &&
T 300 python3 -u tools/step_phases.py > gpurun_out/i_phases_e.log 2>&1 &&
T 400 python3 bench.py --no-cpu-baseline --graphs > gpurun_out/i_bench_g.log 2>&1 &&
T 400 python3 bench.py --no-cpu-baseline > gpurun_out/i_bench_e.log 2>&1
rc=$?
grep "check:" gpurun_out/i_check.log
grep "{" gpurun_out/i_phases_g.log gpurun_out/i_phases_e.log
for f in i_bench_g i_bench_e; do python3 -c "
import json
for l in open('gpurun_out/$f.log'):
    if l.startswith('{'):
        d=json.loads(l); print('$f', round(d['value'],2), 'img/s', round(d['ms_per_step'],1), 'ms', d['step_ms'], 'loss', d['loss'])
" || true; done
exit $rc
