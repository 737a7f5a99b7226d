# SQ counters of the encoder-shape MSDA kernels (one --pmc pass, 8 SQ counters)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
    SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS --kernel-trace --output-format csv -d /tmp/enc_pmc -o run -- \
    python3 "$GRAFT_REPO_ROOT/tools/enc_pmc.py" > "$GRAFT_REPO_ROOT/gpurun_out/p_enc_pmc.log" 2>&1
rc=$?
cd "$GRAFT_REPO_ROOT"
f=$(find /tmp/enc_pmc -name '*counter_collection.csv' | head -n 1)
[ -n "$f" ] && cp "$f" gpurun_out/p_enc_counters.csv
tail -2 gpurun_out/p_enc_pmc.log
exit $rc
