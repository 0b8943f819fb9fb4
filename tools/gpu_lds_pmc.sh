#!/bin/bash
# LDS bank-conflict attribution in k_scan_p4m: one
# rocprofv3 --pmc pass per measurement-build variant of the configs[1] batch
# (MQVS_P4M_DIAG: 0 = as shipped, 8 = the round-5 lane-major walk scratch,
# 4 = no threshold tests / walks, 6 = no tests and no LDS-DMA), counters only.
#   bash tools/gpu_lds_pmc.sh [diag ...]    -> gpurun_out/r06/lds/
set -o pipefail
R="$GRAFT_REPO_ROOT"
O="$R/gpurun_out/r06/lds"
mkdir -p "$O"
cd /tmp || exit 1
export TMPDIR=/tmp
for dg in "${@:-0 8 4 6}"; do
  export MQVS_P4M_DIAG=$dg
  timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES --output-format csv \
    -d "$O/diag$dg" -o run -- python "$R/tools/pmc_search.py" --dbg --searches 2 > "$O/diag$dg.log" 2>&1 \
    || { echo "pmc diag $dg failed"; tail -5 "$O/diag$dg.log"; exit 1; }
  echo "== diag $dg"
  python "$R/tools/pmc_summary.py" k_scan_p4m $(find "$O/diag$dg" -name "*counter_collection.csv") | tee "$O/diag$dg.txt"
done
