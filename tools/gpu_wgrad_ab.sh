# fp32-output weight gradient for the small Linears: GPU tests, then the
# train-step bench with and without it (A/B), then the full GPU suite
set -o pipefail
mkdir -p gpurun_out
T() { timeout -k 10 "$@"; }
T 300 python3 -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
    -k "small_linear or token_linear or wgrad" > gpurun_out/w_tests.log 2>&1 &&
T 300 python3 bench.py --no-cpu-baseline > gpurun_out/w_bench_on.log 2>&1 &&
GDINO_FP32_WGRAD=0 T 300 python3 bench.py --no-cpu-baseline > gpurun_out/w_bench_off.log 2>&1 &&
T 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/w_gpu_tests.log 2>&1
rc=$?
tail -2 gpurun_out/w_tests.log gpurun_out/w_gpu_tests.log
for f in gpurun_out/w_bench_on.log gpurun_out/w_bench_off.log; do
  python3 -c "import json,sys; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); print('$f', d['value'], d['ms_per_step'])" || true
done
exit $rc
