# round 6 GPU sessions: gpurun --timeout 1200 -- bash tools/gpu_r06.sh <mode>
# every GPU step under its own time limit, chained with && (the first
# failure ends the call; no retries)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
T() { timeout -k 10 "$@"; }
step() { echo "[$(date +%T)] $*"; }
PROF=/tmp/gd_prof
MODE="${1:-a}"
PMC_A="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"
PMC_B="SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"

mfma_pmc() {  # tag, microbench args...
  local tag=$1; shift
  step "attn microbench ($tag)" &&
  T 300 python3 tools/attn_microbench.py "$@" > gpurun_out/${tag}_mb.jsonl 2>&1 &&
  step "pmc A ($tag)" &&
  T 240 rocprofv3 --pmc $PMC_A --kernel-trace --output-format csv -d "$PROF/${tag}_a" -o run -- \
      python3 tools/attn_microbench.py --iters 3 --warmup 1 "$@" > gpurun_out/${tag}_pmc_a.log 2>&1 &&
  step "pmc B ($tag)" &&
  T 240 rocprofv3 --pmc $PMC_B --kernel-trace --output-format csv -d "$PROF/${tag}_b" -o run -- \
      python3 tools/attn_microbench.py --iters 3 --warmup 1 "$@" > gpurun_out/${tag}_pmc_b.log 2>&1 &&
  python3 tools/mfma_counters.py --pass "$PROF/${tag}_a" --pass "$PROF/${tag}_b" --bench gpurun_out/${tag}_mb.jsonl \
      --note "$tag" --out gpurun_out/${tag}_mfma_counters.json > gpurun_out/${tag}_mfma_counters.txt 2>&1
}

case "$MODE" in
a)
  # baseline of the round: GPU suite, smoke, driver bench, MFMA counters
  step "pytest -m gpu" &&
  T 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/a_gpu_tests.log 2>&1 &&
  step "smoke" &&
  T 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/a_smoke.log 2>&1 &&
  step "bench (driver command)" &&
  T 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/a_bench.log 2>&1 &&
  mfma_pmc a
  ;;
mb)
  mfma_pmc mb "${@:2}"
  ;;
attn)
  # attention-family parity on the GPU, then the microbench + counters
  step "pytest attention" &&
  T 600 python3 -u -m pytest tests/test_kernels_gpu.py tests/test_blocks_gpu.py -m gpu -x -q --timeout 120 \
      --timeout-method thread -k "attention or block" > gpurun_out/attn_tests.log 2>&1 &&
  mfma_pmc attn --cases attn
  ;;
kern)
  # attention + window-attention parity on the GPU, then microbench + counters
  step "pytest attention / window / blocks" &&
  T 600 python3 -u -m pytest tests/test_kernels_gpu.py tests/test_blocks_gpu.py -m gpu -x -q --timeout 120 \
      --timeout-method thread -k "attention or block or swin" > gpurun_out/kern_tests.log 2>&1 &&
  mfma_pmc kern --cases attn,wattn
  ;;
margins)
  # the kernel parity tests with north_star's flat tolerances, every check
  # recorded (no -x: all margins in one pass), then the MSDA tests
  step "pytest kernels (margins)"
  GD_MARGINS=gpurun_out/kernel_margins.jsonl T 900 python3 -u -m pytest tests/test_kernels_gpu.py -m gpu -q \
      --timeout 120 --timeout-method thread > gpurun_out/margins_tests.log 2>&1
  rc1=$?
  [ $rc1 -eq 0 ] || [ $rc1 -eq 1 ] || exit $rc1
  step "pytest msda" &&
  T 600 python3 -u -m pytest tests/test_msda_gpu.py -m gpu -q --timeout 120 --timeout-method thread \
      > gpurun_out/msda_tests.log 2>&1
  ;;
km)
  # margins (all kernel parity checks recorded), MSDA parity, block goldens,
  # then the attention / window microbench + counters
  step "pytest kernels (margins)"
  GD_MARGINS=gpurun_out/kernel_margins.jsonl T 900 python3 -u -m pytest tests/test_kernels_gpu.py -m gpu -q \
      --timeout 120 --timeout-method thread > gpurun_out/margins_tests.log 2>&1
  rc1=$?
  [ $rc1 -eq 0 ] || [ $rc1 -eq 1 ] || exit $rc1
  step "pytest msda + blocks" &&
  T 600 python3 -u -m pytest tests/test_msda_gpu.py tests/test_blocks_gpu.py -m gpu -q --timeout 120 \
      --timeout-method thread > gpurun_out/msda_tests.log 2>&1
  rc2=$?
  [ $rc2 -eq 0 ] || [ $rc2 -eq 1 ] || exit $rc2
  mfma_pmc kern --cases attn,wattn
  ;;
km2)
  # margins + MSDA / block parity, kernel microbench + counters, decoder
  # MSDA backward variants, the driver's bench command
  step "pytest kernels (margins)"
  GD_MARGINS=gpurun_out/kernel_margins.jsonl T 900 python3 -u -m pytest tests/test_kernels_gpu.py -m gpu -q \
      --timeout 120 --timeout-method thread > gpurun_out/margins_tests.log 2>&1
  rc1=$?
  [ $rc1 -eq 0 ] || [ $rc1 -eq 1 ] || exit $rc1
  step "pytest msda + blocks" &&
  T 600 python3 -u -m pytest tests/test_msda_gpu.py tests/test_blocks_gpu.py -m gpu -q --timeout 120 \
      --timeout-method thread > gpurun_out/msda_tests.log 2>&1
  rc2=$?
  [ $rc2 -eq 0 ] || [ $rc2 -eq 1 ] || exit $rc2
  mfma_pmc kern --cases attn,wattn &&
  step "msda decoder-shape backward variants" &&
  T 300 python3 tools/msda_microbench.py --bwd-variants --geom dec --variant "lane32,sorted-all,sorted F1,sorted F4" \
      > gpurun_out/decmsda.jsonl 2>&1 &&
  step "bench (driver command)" &&
  T 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench.log 2>&1
  ;;
r6d)
  # add+LayerNorm vector kernels and the window-attention block heuristic:
  # parity, window microbench A/B, the driver's bench, kernel census trace
  step "pytest norm / window / blocks / stepgraph" &&
  T 900 python3 -u -m pytest tests/test_kernels_gpu.py tests/test_blocks_gpu.py tests/test_stepgraph_gpu.py -m gpu -q \
      --timeout 120 --timeout-method thread -k "norm or window or block or swin or step" > gpurun_out/r6d_tests.log 2>&1 &&
  step "wattn microbench (blocks 1024 / 2048)" &&
  T 300 python3 tools/attn_microbench.py --cases wattn > gpurun_out/r6d_wattn_1024.jsonl 2>&1 &&
  GD_WATTN_BLOCKS=2048 T 300 python3 tools/attn_microbench.py --cases wattn > gpurun_out/r6d_wattn_2048.jsonl 2>&1 &&
  step "bench (driver command)" &&
  T 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r6d_bench.log 2>&1 &&
  step "census trace" &&
  T 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$PROF/r6d_prof" -o run -- \
      python3 bench.py --no-cpu-baseline --steps 4 --warmup 3 --ckpt-compare off > gpurun_out/r6d_prof.log 2>&1 &&
  kt=$(find "$PROF/r6d_prof" -name '*kernel_trace.csv' | head -n 1) &&
  python3 tools/trace_steps.py --skip 2 "$kt" > gpurun_out/r6d_steady_state.txt 2>&1
  ;;
r6e)
  # window attention with LDS-only in-loop barriers: parity, microbench,
  # then the census (below)
  step "pytest window / blocks" &&
  T 900 python3 -u -m pytest tests/test_kernels_gpu.py tests/test_blocks_gpu.py -m gpu -q \
      --timeout 120 --timeout-method thread -k "window or block or swin" > gpurun_out/r6e_tests.log 2>&1 &&
  step "wattn microbench" &&
  T 300 python3 tools/attn_microbench.py --cases wattn > gpurun_out/r6e_wattn.jsonl 2>&1 &&
  step "census trace" &&
  T 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$PROF/census" -o run -- \
      python3 bench.py --no-cpu-baseline --steps 4 --warmup 3 --ckpt-compare off > gpurun_out/census_prof.log 2>&1 &&
  kt=$(find "$PROF/census" -name '*kernel_trace.csv' | head -n 1) &&
  python3 tools/trace_steps.py --skip 2 "$kt" > gpurun_out/census_steady_state.txt 2>&1 &&
  step "glue census (all ops)" &&
  T 300 python3 tools/glue_census.py --min-numel 1 --out gpurun_out/census_glue_all.txt > gpurun_out/census_glue.log 2>&1
  ;;
tlx)
  # x-resident token-linear kernel: parity, then shapes A/B against the
  # chunked kernel and the library GEMM
  step "pytest token linear / blocks" &&
  T 600 python3 -u -m pytest tests/test_kernels_gpu.py tests/test_blocks_gpu.py -m gpu -q --timeout 120 \
      --timeout-method thread -k "linear or tlin or block or ffn" > gpurun_out/tlx_tests.log 2>&1 &&
  step "tlin microbench" &&
  T 300 python3 tools/tlin_microbench.py > gpurun_out/tlx_mb.jsonl 2>&1
  ;;
fin)
  # the round's final evidence: the whole GPU suite (kernel margins recorded),
  # smoke, microbenchmarks, the driver's bench, then the rocprofv3 trace and
  # the FETCH_SIZE / WRITE_SIZE passes of the same step (one counter per run)
  step "pytest -m gpu (margins recorded)"
  GD_MARGINS=gpurun_out/fin_kernel_margins.jsonl T 600 python3 -u -m pytest tests -m gpu -q --timeout 120 \
      --timeout-method thread > gpurun_out/fin_gpu_tests.log 2>&1
  rc1=$?
  [ $rc1 -eq 0 ] || [ $rc1 -eq 1 ] || exit $rc1
  step "smoke" &&
  T 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin_smoke.log 2>&1 &&
  step "microbenchmarks" &&
  T 200 python3 tools/tlin_microbench.py > gpurun_out/fin_tlin.jsonl 2>&1 &&
  T 200 python3 tools/attn_microbench.py --cases attn,wattn > gpurun_out/fin_attn_mb.jsonl 2>&1 &&
  step "bench (driver command)" &&
  T 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/fin_bench.log 2>&1 &&
  step "rocprof kernel trace" &&
  T 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PROF/fin_prof" -o run -- \
      python3 bench.py --no-cpu-baseline --steps 4 --warmup 3 --ckpt-compare off > gpurun_out/fin_prof.log 2>&1 &&
  mkdir -p gpurun_out/fin_prof &&
  find "$PROF/fin_prof" -name '*stats*.csv' -exec cp {} gpurun_out/fin_prof/ \; &&
  kt=$(find "$PROF/fin_prof" -name '*kernel_trace.csv' | head -n 1) &&
  python3 tools/trace_steps.py --skip 2 "$kt" > gpurun_out/fin_prof/steady_state.txt 2>&1 &&
  step "pmc FETCH_SIZE" &&
  T 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$PROF/fin_fetch" -o run -- \
      python3 bench.py --no-cpu-baseline --steps 1 --warmup 1 --ckpt-compare off > gpurun_out/fin_fetch.log 2>&1 &&
  step "pmc WRITE_SIZE" &&
  T 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$PROF/fin_write" -o run -- \
      python3 bench.py --no-cpu-baseline --steps 1 --warmup 1 --ckpt-compare off > gpurun_out/fin_write.log 2>&1 &&
  python3 tools/pmc_traffic.py --fetch "$PROF/fin_fetch" --write "$PROF/fin_write" \
      --out gpurun_out/fin_pmc_traffic.json > gpurun_out/fin_pmc_traffic.log 2>&1 &&
  exit $rc1
  ;;
fin2)
  # after the last host-side launch trims: the GPU suite, the driver's bench
  # and the graph-step census
  step "pytest -m gpu"
  T 600 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/fin2_gpu_tests.log 2>&1
  rc1=$?
  [ $rc1 -eq 0 ] || [ $rc1 -eq 1 ] || exit $rc1
  step "bench (driver command)" &&
  T 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/fin2_bench.log 2>&1 &&
  step "census trace" &&
  T 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PROF/fin2" -o run -- \
      python3 bench.py --no-cpu-baseline --steps 4 --warmup 3 --ckpt-compare off > gpurun_out/fin2_prof.log 2>&1 &&
  kt=$(find "$PROF/fin2" -name '*kernel_trace.csv' | head -n 1) &&
  python3 tools/trace_steps.py --skip 2 "$kt" > gpurun_out/fin2_steady_state.txt 2>&1 &&
  exit $rc1
  ;;
benchab)
  # the default of every round-6 A/B switch against its alternative, the
  # driver's bench (checkpointing compare off) per setting
  for sw in BASE GD_ATTN_SPLIT=0 GD_WATTN_BWD2=0 GD_ADDLN_V4=0 GD_TLIN=0 GD_WATTN_BLOCKS=2048 BASE2; do
    step "bench with $sw"
    case "$sw" in BASE*) e=() ;; *) e=("$sw") ;; esac
    env "${e[@]}" timeout -k 10 300 python3 bench.py --no-cpu-baseline --ckpt-compare off --steps 20 --warmup 5 \
        > "gpurun_out/benchab_${sw%%=*}.log" 2>&1 || exit $?
    grep '^{' "gpurun_out/benchab_${sw%%=*}.log" | tail -1 | cut -c1-120
  done
  ;;
knobs)
  # the driver's bench (checkpointing compare off) under each NAME=VALUE
  # given after the mode, BASE = the defaults
  for sw in "${@:2}"; do
    step "bench with $sw"
    case "$sw" in BASE*) e=() ;; *) e=("$sw") ;; esac
    env "${e[@]}" timeout -k 10 300 python3 bench.py --no-cpu-baseline --ckpt-compare off --steps 20 --warmup 5 \
        > "gpurun_out/knobs_${sw//[=,]/_}.log" 2>&1 || exit $?
    grep '^{' "gpurun_out/knobs_${sw//[=,]/_}.log" | tail -1 | cut -c60-130
  done
  ;;
prof)
  # the final build's rocprofv3 --stats trace and FETCH_SIZE / WRITE_SIZE
  # passes of the bench step (one counter per run)
  step "rocprof kernel trace" &&
  T 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PROF/prof" -o run -- \
      python3 bench.py --no-cpu-baseline --steps 4 --warmup 3 --ckpt-compare off > gpurun_out/prof_trace.log 2>&1 &&
  mkdir -p gpurun_out/prof &&
  find "$PROF/prof" -name '*stats*.csv' -exec cp {} gpurun_out/prof/ \; &&
  kt=$(find "$PROF/prof" -name '*kernel_trace.csv' | head -n 1) &&
  python3 tools/trace_steps.py --skip 2 "$kt" > gpurun_out/prof/steady_state.txt 2>&1 &&
  step "pmc FETCH_SIZE" &&
  T 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$PROF/prof_fetch" -o run -- \
      python3 bench.py --no-cpu-baseline --steps 1 --warmup 1 --ckpt-compare off > gpurun_out/prof_fetch.log 2>&1 &&
  step "pmc WRITE_SIZE" &&
  T 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$PROF/prof_write" -o run -- \
      python3 bench.py --no-cpu-baseline --steps 1 --warmup 1 --ckpt-compare off > gpurun_out/prof_write.log 2>&1 &&
  python3 tools/pmc_traffic.py --fetch "$PROF/prof_fetch" --write "$PROF/prof_write" \
      --out gpurun_out/prof_pmc_traffic.json > gpurun_out/prof_pmc_traffic.log 2>&1
  ;;
lossab)
  # which round-6 kernel change moved cfg3's bf16 loss error: the full-size
  # gradient test under each A/B switch (one process per setting)
  for sw in BASE GD_ATTN_SPLIT=0 GD_WATTN_BWD2=0 GD_ADDLN_V4=0 GD_TLIN=0; do
    step "cfg3 with $sw"
    if [ "$sw" = BASE ]; then e=(); else e=("$sw"); fi
    env "${e[@]}" timeout -k 10 300 python3 -u -m pytest tests/test_fullsize_gpu.py -m gpu -q -s --timeout 240 \
        --timeout-method thread -k cfg3_gradients > "gpurun_out/lossab_${sw%%=*}.log" 2>&1
    rc=$?
    [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
    grep -E "loss:|pred_logits:|q0.5" "gpurun_out/lossab_${sw%%=*}.log"
  done
  ;;
census)
  step "census trace" &&
  T 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$PROF/census" -o run -- \
      python3 bench.py --no-cpu-baseline --steps 4 --warmup 3 --ckpt-compare off > gpurun_out/census_prof.log 2>&1 &&
  kt=$(find "$PROF/census" -name '*kernel_trace.csv' | head -n 1) &&
  python3 tools/trace_steps.py --skip 2 "$kt" > gpurun_out/census_steady_state.txt 2>&1 &&
  step "glue census (all ops)" &&
  T 300 python3 tools/glue_census.py --min-numel 1 --out gpurun_out/census_glue_all.txt > gpurun_out/census_glue.log 2>&1
  ;;
decmsda)
  step "msda decoder-shape backward variants" &&
  T 300 python3 tools/msda_microbench.py --bwd-variants --geom dec --variant "lane32,sorted-all,sorted F1,sorted F4" \
      > gpurun_out/decmsda.jsonl 2>&1
  ;;
bench)
  step "bench (driver command)" &&
  T 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1
  ;;
*)
  echo "usage: $0 a|mb|bench" >&2; exit 2 ;;
esac
rc=$?
step "done rc=$rc"
exit $rc
