set -o pipefail
mkdir -p gpurun_out
T() { timeout -k 10 "$@"; }
T 400 python3 bench.py > gpurun_out/k_bench.log 2>&1 || exit $?
T 300 python3 -u -m pytest tests/test_msda_gpu.py -x -q --timeout 120 --timeout-method thread -k "sorted or pixel_block or init_geometry" > gpurun_out/k_msda.log 2>&1
rc=$?
tail -2 gpurun_out/k_msda.log
python3 -c "
import json
for l in open('gpurun_out/k_bench.log'):
    if l.startswith('{'):
        d=json.loads(l); print(round(d['value'],2), 'img/s', round(d['ms_per_step'],1), 'ms', d.get('step_ms'), d['roofline'], d['options'], d['kernels'])
"
exit $rc
