# round-3 check: eager vs graph loss trajectories after the cast-cache fix,
# then the eager and graph bench lines (driver command shape)
set -o pipefail
mkdir -p gpurun_out
T() { timeout -k 10 "$@"; }
T 600 python3 -u tools/graph_probe.py traj > gpurun_out/a_traj.log 2>&1 &&
T 400 python3 bench.py --no-cpu-baseline > gpurun_out/a_bench_eager.log 2>&1 &&
T 400 python3 bench.py --no-cpu-baseline --graphs > gpurun_out/a_bench_graphs.log 2>&1
rc=$?
grep losses gpurun_out/a_traj.log
for f in a_bench_eager a_bench_graphs; do python3 -c "
import json,sys
for l in open('gpurun_out/$f.log'):
    if l.startswith('{'):
        d=json.loads(l); print('$f', round(d['value'],2), 'img/s', round(d['ms_per_step'],1), 'ms', d['step_ms'], 'loss', d['loss'])
" || true; done
exit $rc
