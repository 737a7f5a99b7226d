#!/usr/bin/env bash
# One GPU session on a fresh MI355X box (run through gpurun from the repo root):
#   gpurun --timeout 1200 -- bash tools/gpu_session.sh <mode>
# Every GPU step has its own time limit and the steps are chained with &&:
# the first failure ends the session (no retries, no further GPU work).
# Small logs go to gpurun_out/ (merged back, <= 64 MiB); raw profiler output
# stays in /tmp on the box and only its summaries are copied to gpurun_out/.
set -euo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
MODE="${1:-core}"
T() { timeout -k 10 "$@"; }
step() { echo "[$(date +%T)] $*"; }
PROF=/tmp/gd_prof

# rocprofv3 kernel trace of a short bench run; summaries only
prof_trace() {  # name, bench args...
  local name=$1; shift
  step "rocprof kernel trace: $name"
  T 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$PROF/$name" -o run -- \
      python3 bench.py --no-cpu-baseline "$@" > "gpurun_out/${name}.log" 2>&1
  mkdir -p "gpurun_out/$name"
  find "$PROF/$name" -name '*stats*.csv' -exec cp {} "gpurun_out/$name/" \;
  local kt; kt=$(find "$PROF/$name" -name '*kernel_trace.csv' | head -n 1 || true)
  if [ -n "$kt" ]; then
    python3 tools/trace_steps.py --skip 2 "$kt" > "gpurun_out/$name/steady_state.txt" 2>&1 || true
    if [ "${KEEP_TRACE:-0}" = 1 ]; then gzip -c "$kt" > "gpurun_out/$name/kernel_trace.csv.gz"; fi
  fi
}
# one PMC pass (one counter group per run)
prof_pmc() {  # name, counters, bench args...
  local name=$1 counters=$2; shift 2
  step "rocprof pmc $counters: $name"
  T 600 rocprofv3 --pmc $counters --kernel-trace --output-format csv -d "$PROF/$name" -o run -- \
      python3 bench.py --no-cpu-baseline "$@" > "gpurun_out/${name}.log" 2>&1
}

case "$MODE" in
tests)
  step "pytest -m gpu"
  T 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
      > gpurun_out/s_gpu_tests.log 2>&1
  ;;
bench)
  step "bench (default)"
  T 600 python3 bench.py > gpurun_out/s_bench.log 2>&1 && tail -c 600 gpurun_out/s_bench.log
  ;;
core)
  # parity, the default bench line, A/B of the encoder backward, the kernel
  # trace, and HBM traffic counters in their own passes (FETCH_SIZE and
  # WRITE_SIZE do not fit one TCC pass; MI355X_MICROARCH.md "rocprofv3 PMC")
  step "pytest -m gpu"
  T 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
      > gpurun_out/s_gpu_tests.log 2>&1 &&
  step "bench (default)" &&
  T 600 python3 bench.py > gpurun_out/s_bench.log 2>&1 &&
  step "bench (lane32 encoder backward, A/B)" &&
  GD_MSDA_BWD=lane32 T 600 python3 bench.py --no-cpu-baseline > gpurun_out/s_bench_lane32.log 2>&1 &&
  step "bench (forward only, config 2)" &&
  T 600 python3 bench.py --no-cpu-baseline --forward-only > gpurun_out/s_bench_fwd.log 2>&1 &&
  prof_trace s_prof --steps 3 --warmup 2 &&
  prof_pmc s_pmc_fetch FETCH_SIZE --steps 1 --warmup 1 &&
  prof_pmc s_pmc_write WRITE_SIZE --steps 1 --warmup 1 &&
  step "pmc_traffic" &&
  python3 tools/pmc_traffic.py --fetch "$PROF/s_pmc_fetch" --write "$PROF/s_pmc_write" \
      --out gpurun_out/s_pmc_traffic.json > gpurun_out/s_pmc_traffic.log 2>&1
  ;;
final)
  # MSDA forward batching variants, parity, the default and forward-only
  # bench lines, trace + PMC passes
  step "pytest -m gpu"
  T 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
      > gpurun_out/s_gpu_tests.log 2>&1 &&
  step "bench (default)" &&
  T 600 python3 bench.py > gpurun_out/s_bench.log 2>&1 &&
  step "bench (forward only, config 2)" &&
  T 600 python3 bench.py --no-cpu-baseline --forward-only > gpurun_out/s_bench_fwd.log 2>&1 &&
  prof_trace s_prof --steps 3 --warmup 2 &&
  prof_pmc s_pmc_fetch FETCH_SIZE --steps 1 --warmup 1 &&
  prof_pmc s_pmc_write WRITE_SIZE --steps 1 --warmup 1 &&
  step "pmc_traffic" &&
  python3 tools/pmc_traffic.py --fetch "$PROF/s_pmc_fetch" --write "$PROF/s_pmc_write" \
      --out gpurun_out/s_pmc_traffic.json > gpurun_out/s_pmc_traffic.log 2>&1
  ;;
benchprof)
  # the driver's bench command, then the trace + PMC passes of the same step
  step "bench (driver command)"
  T 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/s_bench.log 2>&1 &&
  prof_trace s_prof --steps 3 --warmup 2 &&
  prof_pmc s_pmc_fetch FETCH_SIZE --steps 1 --warmup 1 &&
  prof_pmc s_pmc_write WRITE_SIZE --steps 1 --warmup 1 &&
  step "pmc_traffic" &&
  python3 tools/pmc_traffic.py --fetch "$PROF/s_pmc_fetch" --write "$PROF/s_pmc_write" \
      --out gpurun_out/s_pmc_traffic.json > gpurun_out/s_pmc_traffic.log 2>&1
  ;;
census)
  # kernel census of the default (checkpointing-off) step graph only
  prof_trace s_prof --steps 4 --warmup 3 --ckpt-compare off
  ;;
prof)
  prof_trace s_prof --steps 3 --warmup 2 &&
  prof_pmc s_pmc_fetch FETCH_SIZE --steps 1 --warmup 1 &&
  prof_pmc s_pmc_write WRITE_SIZE --steps 1 --warmup 1 &&
  step "pmc_traffic" &&
  python3 tools/pmc_traffic.py --fetch "$PROF/s_pmc_fetch" --write "$PROF/s_pmc_write" \
      --out gpurun_out/s_pmc_traffic.json > gpurun_out/s_pmc_traffic.log 2>&1
  ;;
ab)
  # A/B of every kernel family against its torch composition (GDINO_DISABLE)
  T 600 python3 bench.py --no-cpu-baseline > gpurun_out/s_ab_all.log 2>&1 &&
  for fam in wattn attn contrastive prologue wgrad addln; do
    GDINO_DISABLE=$fam T 600 python3 bench.py --no-cpu-baseline > "gpurun_out/s_ab_no_$fam.log" 2>&1 || exit $?
  done &&
  GDINO_DISABLE=wattn,attn,contrastive,prologue,wgrad,addln T 600 python3 bench.py --no-cpu-baseline \
      > gpurun_out/s_ab_none.log 2>&1
  ;;
graphs)
  # HIP-graph replay (experimental): run alone, in its own gpurun call
  GDINO_GRAPH_DEBUG=1 T 600 python3 bench.py --no-cpu-baseline --graphs --steps 5 --warmup 2 \
      > gpurun_out/s_bench_graphs.log 2>&1
  ;;
msdapmc)
  # encoder-shape MSDA kernels alone: timings per variant, then FETCH_SIZE
  # and WRITE_SIZE in separate --pmc passes over tools/enc_pmc.py
  step "msda microbench (sorted backward, encoder shapes)" &&
  T 300 python3 tools/msda_microbench.py --bwd-variants --variant sorted > gpurun_out/s_msda_bwd.jsonl 2>&1 &&
  step "pmc FETCH_SIZE" &&
  T 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --kernel-include-regex "msda|scan|fill" --output-format csv \
      -d "$PROF/m_fetch" -o run -- python3 tools/enc_pmc.py > gpurun_out/s_pmc_fetch.log 2>&1 &&
  step "pmc WRITE_SIZE" &&
  T 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --kernel-include-regex "msda|scan|fill" --output-format csv \
      -d "$PROF/m_write" -o run -- python3 tools/enc_pmc.py > gpurun_out/s_pmc_write.log 2>&1 &&
  python3 tools/pmc_traffic.py --fetch "$PROF/m_fetch" --write "$PROF/m_write" \
      --out gpurun_out/s_pmc_traffic.json > gpurun_out/s_pmc_traffic.log 2>&1
  ;;
syncab)
  # the driver's bench command with the device-wide sync after each replay and
  # with the event-bounded replay queue
  step "bench (device sync)" &&
  GDINO_STEPGRAPH_SYNC=device T 600 python3 bench.py --no-cpu-baseline > gpurun_out/s_bench_device.log 2>&1 &&
  step "bench (event-bounded)" &&
  GDINO_STEPGRAPH_SYNC=event T 600 python3 bench.py --no-cpu-baseline > gpurun_out/s_bench_event.log 2>&1
  ;;
*)
  echo "usage: $0 [tests|bench|core|prof|ab|graphs|msdapmc|syncab]" >&2
  exit 2
  ;;
esac
rc=$?
step "done rc=$rc"; du -sh gpurun_out
exit $rc
