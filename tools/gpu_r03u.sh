# TunableOp: tune the train step's GEMM shapes (table written under gpurun_out/),
# then the bench with and without the table
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T() { timeout -k 10 "$@"; }
step() { echo "[$(date +%T)] $*"; }
step tune
T 900 python3 -u tools/tune_gemms.py --out gpurun_out/gdino_train_gfx950.csv --ms 20 > gpurun_out/u_tune.log 2>&1 || exit $?
tail -3 gpurun_out/u_tune.log
step bench-tuned
T 400 python3 bench.py --no-cpu-baseline --tunableop gpurun_out/gdino_train_gfx950.csv > gpurun_out/u_bench_tuned.log 2>&1 || exit $?
step bench-default
T 400 python3 bench.py --no-cpu-baseline > gpurun_out/u_bench.log 2>&1 || exit $?
for f in u_bench_tuned u_bench; do python3 -c "
import json
for l in open('gpurun_out/$f.log'):
    if l.startswith('{'):
        d=json.loads(l); print('$f', round(d['value'],2), 'img/s', round(d['ms_per_step'],1), 'ms', d['step_ms']['p50'], d['loss'])
"; done
