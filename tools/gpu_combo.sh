# Round-2 final checks, most important first: the whole GPU suite, the
# train-step and forward bench lines, encoder-backward depth / probes, the
# kernel trace and PMC passes of the final build, then the HIP-graph trial
# (the risky step last)
set -o pipefail
mkdir -p gpurun_out
T() { timeout -k 10 "$@"; }
T 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/e_tests.log 2>&1 &&
T 300 python3 bench.py > gpurun_out/w_bench_on.log 2>&1 &&
T 300 python3 bench.py --no-cpu-baseline --forward-only > gpurun_out/w_bench_fwd.log 2>&1 &&
T 300 python3 tools/msda_microbench.py --enc-probes > gpurun_out/e_probes.log 2>&1 &&
bash tools/gpu_session.sh prof &&
bash tools/gpu_graphs.sh
rc=$?
tail -2 gpurun_out/e_tests.log
for f in gpurun_out/w_bench_on.log gpurun_out/w_bench_fwd.log; do
  python3 -c "import json; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); print('$f', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])" || true
done
head -5 gpurun_out/e_probes.log | cut -c1-160
exit $rc
