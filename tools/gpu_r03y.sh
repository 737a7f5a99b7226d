# LDS-histogram coarse-level counting / slot reservation: parity, microbench, per-geometry breakdown
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T() { timeout -k 10 "$@"; }
step() { echo "[$(date +%T)] $*"; }
step parity
T 600 python3 -u -m pytest tests/test_msda_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/y_parity.log 2>&1
rc=$?; tail -2 gpurun_out/y_parity.log; [ $rc -ne 0 ] && exit $rc
step microbench
T 300 python3 tools/msda_microbench.py --bwd-variants --iters 20 > gpurun_out/y_bwd_variants.jsonl 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/y_bwd_variants.jsonl | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['geom'], d['variant'], round(d['bwd_us'], 1))
"
bash tools/gpu_r03x.sh
