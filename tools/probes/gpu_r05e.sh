# round 5: step-graph GPU tests, the bench (protocol + checkpoint-on line),
# then one TunableOp tuning run and the bench on its table
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/test_stepgraph_gpu.py -v --timeout 300 --timeout-method thread > gpurun_out/e_sg.log 2>&1 ;
timeout -k 10 600 python3 bench.py --no-cpu-baseline > gpurun_out/e_bench.log 2>&1 &&
timeout -k 10 900 python3 tools/tune_gemms.py --out gpurun_out/tunableop_gfx950.csv > gpurun_out/e_tune.log 2>&1 &&
timeout -k 10 600 python3 bench.py --no-cpu-baseline --ckpt-compare off --tunableop gpurun_out/tunableop_gfx950.csv > gpurun_out/e_bench_tuned.log 2>&1
