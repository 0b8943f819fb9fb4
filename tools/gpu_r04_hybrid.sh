#!/bin/bash
# configs[4] gathered-scan evidence: PMC passes at 10 % and 1 % selectivity
# (50M x 768 L2, nq 1) and a kernel trace of the 1 % search.
# Outputs gpurun_out/r04_hybrid/.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04_hybrid
mkdir -p $O
STEPS="${*:-pmc trace}"
pmc_set() {  # tag, searches, args...
  local tag=$1 s=$2; shift 2
  bash tools/gpu_pmc.sh python tools/pmc_search.py --searches "$s" "$@" || return 1
  rm -rf "$O/pmc_$tag" && mkdir -p "$O/pmc_$tag" && mv gpurun_out/pmc1 gpurun_out/pmc2 gpurun_out/pmc3 gpurun_out/pmc*.log "$O/pmc_$tag/" || return 1
}
for step in $STEPS; do
  case $step in
    pmc)
      for sel in 10 1; do
        pmc_set sel$sel 4 --nq 1 --n 50000000 --metric L2 --selectivity $sel || exit 1
        python tools/pmc_traffic.py $O/pmc_sel$sel --searches 5 --nq 1 --kernel "k_(?:scan|chunk_count|pad_scan|compact|probe|survivors|exact|sort|refine)" \
          --out $O/pmc_config4_sel$sel.json > /dev/null || exit 1
        echo "== sel $sel"; grep -E '"k_|hbm_bytes_per_search|avg_launch' $O/pmc_config4_sel$sel.json
      done ;;
    trace)
      ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/trace1" -o run --output-format csv \
          -- python3 "$GRAFT_REPO_ROOT/tools/pmc_search.py" --nq 1 --n 50000000 --metric L2 --selectivity 1 --searches 4 \
          > "$GRAFT_REPO_ROOT/$O/trace1.log" 2>&1 ) || { echo "trace failed"; tail -5 $O/trace1.log; exit 1; }
      python3 tools/timeline.py $O/trace1/run_kernel_trace.csv --start k_chunk_count --nth -1 ;;
  esac
done
exit 0
