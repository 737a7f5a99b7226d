# Per-family A/B (each HIP kernel family against its torch composition) and
# a BASELINE config-5 line (Swin-B/384 backbone at 1024x1024, bs=2); every
# step has its own limit and the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
T() { timeout -k 10 "$@"; }
T 300 python3 bench.py --no-cpu-baseline --backbone swin_B_384_22k --height 1024 --width 1024 \
    > gpurun_out/f_cfg5.log 2>&1 &&
T 300 python3 bench.py --no-cpu-baseline > gpurun_out/f_ab_all.log 2>&1 &&
for fam in wattn attn contrastive prologue wgrad addln; do
  GDINO_DISABLE=$fam T 300 python3 bench.py --no-cpu-baseline > "gpurun_out/f_ab_no_$fam.log" 2>&1 || exit $?
done &&
GDINO_DISABLE=wattn,attn,contrastive,prologue,wgrad,addln T 300 python3 bench.py --no-cpu-baseline \
    > gpurun_out/f_ab_none.log 2>&1
rc=$?
for f in gpurun_out/f_*.log; do
  python3 -c "import json; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); print('$f', round(d['value'],2), round(d['ms_per_step'],1))" || true
done
exit $rc
