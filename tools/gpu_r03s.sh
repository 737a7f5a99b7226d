# HBM traffic of the MSDA kernels: separate FETCH_SIZE / WRITE_SIZE passes,
# counters collected for the MSDA / scan kernels only, eager step
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp
R=$GRAFT_REPO_ROOT
step() { echo "[$(date +%T)] $*"; }
for c in FETCH_SIZE WRITE_SIZE; do
  step "pmc $c"
  timeout -s KILL 240 rocprofv3 --pmc $c --kernel-include-regex "msda|scan_" --kernel-trace --output-format csv -d /tmp/pmc_$c -o run -- python3 $R/bench.py --no-cpu-baseline --no-graphs --steps 1 --warmup 1 > $R/gpurun_out/s_pmc_$c.log 2>&1 || exit $?
done
step pmc_traffic
cd $R && python3 tools/pmc_traffic.py --fetch /tmp/pmc_FETCH_SIZE --write /tmp/pmc_WRITE_SIZE --out gpurun_out/s_pmc_traffic.json > gpurun_out/s_pmc_traffic.log 2>&1
cat gpurun_out/s_pmc_traffic.log
