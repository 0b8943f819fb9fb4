#!/bin/bash
# L2 behaviour of one pre-filter scan config (rocprofv3 --pmc passes, counters
# only): bash tools/gpu_pmc_mx.sh TAG "mx:default" [extra tune_bf16.py args]
# Writes gpurun_out/pmcmx_TAG{1,2,3}/.
set -o pipefail
R="$GRAFT_REPO_ROOT"
TAG=$1; CFG=$2; shift 2
cd /tmp || exit 1
export TMPDIR=/tmp
mkdir -p "$R/gpurun_out"
run() {
    local tag=$1; shift
    timeout -k 10 150 rocprofv3 --pmc "$@" --output-format csv -d "$R/gpurun_out/$tag" -o run \
        -- python3 "$R/tools/tune_bf16.py" --configs "$CFG" --rounds 1 "${EXTRA[@]}" > "$R/gpurun_out/$tag.log" 2>&1
}
EXTRA=("$@")
run pmcmx_${TAG}1 TCC_HIT_sum TCC_MISS_sum SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
    && run pmcmx_${TAG}2 FETCH_SIZE \
    && run pmcmx_${TAG}3 GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS
rc=$?
echo "pmc rc=$rc"
exit $rc
