#!/bin/bash
# PMC passes (each its own rocprofv3 run, counters only -- no trace domains)
# over a command given as arguments, e.g.
#   bash tools/gpu_pmc.sh python tools/tune_bf16.py --vars 0,7 --rounds 1
# Writes gpurun_out/pmc{1,2,3}/.
set -o pipefail
R="$GRAFT_REPO_ROOT"
cd /tmp || exit 1
export TMPDIR=/tmp
mkdir -p "$R/gpurun_out"
run() {
    local tag=$1; shift
    timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d "$R/gpurun_out/$tag" -o run \
        -- "${CMD[@]}" > "$R/gpurun_out/$tag.log" 2>&1
}
CMD=("$@")
CMD[1]="$R/${CMD[1]}"
run pmc1 GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS \
    && run pmc2 FETCH_SIZE \
    && run pmc3 WRITE_SIZE TCC_HIT_sum TCC_MISS_sum SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE
rc=$?
echo "pmc rc=$rc"
find "$R/gpurun_out" -path "*pmc*" -name "*counter_collection*"
exit $rc
