# round 5: bench A/B of the geometry-shared MSDA kernels in the real step
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in "1 1" "0 0" "1 0" "0 1"; do
  set -- $v
  GD_MSDA_FWD_GS=$1 GD_MSDA_SORTED_GS=$2 timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 8 --no-cpu-baseline --ckpt-compare off > gpurun_out/i_fwd$1_bwd$2.json 2> gpurun_out/i_fwd$1_bwd$2.err || exit $?
done
