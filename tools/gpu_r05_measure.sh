#!/bin/bash
# Round-5 measurement session: PMC passes for the headline batch (configs[1]),
# nq = 1 and configs[4] at 100 % selectivity; the BLAS-order risk count; then
# the bench line and its rocprofv3 kernel-trace summary.  Every GPU step has its
# own time limit; the first failure ends the session.  Outputs under
# gpurun_out/r05/.
#   bash tools/gpu_r03_measure.sh [pmc|risk|bench]...   (default: all three)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05
mkdir -p $O
STEPS="${*:-pmc pmc4 index bench}"
pmc_set() {  # tag, searches, args...
  local tag=$1 s=$2; shift 2
  bash tools/gpu_pmc.sh python tools/pmc_search.py --searches "$s" "$@" || return 1
  rm -rf "$O/pmc_$tag" && mkdir -p "$O/pmc_$tag" && mv gpurun_out/pmc1 gpurun_out/pmc2 gpurun_out/pmc3 gpurun_out/pmc*.log "$O/pmc_$tag/" || return 1
}
for step in $STEPS; do
  case $step in
    pmc)
      pmc_set config1 2 --nq 1000 || exit 1
      python tools/pmc_traffic.py $O/pmc_config1 --searches 3 --nq 1000 --out $O/pmc_traffic.json > /dev/null || exit 1
      pmc_set nq1 4 --nq 1 || exit 1
      python tools/pmc_traffic.py $O/pmc_nq1 --searches 5 --nq 1 --out $O/pmc_nq1.json > /dev/null || exit 1
      echo "pmc done"; cat $O/pmc_traffic.json $O/pmc_nq1.json | grep -E "hbm_bytes_per_search|avg_launch|clock|mfma_busy|k_scan" ;;
    pmc4)
      pmc_set config4 4 --nq 1 --n 50000000 --metric L2 --selectivity 100 || exit 1
      python tools/pmc_traffic.py $O/pmc_config4 --searches 5 --nq 1 --out $O/pmc_config4_sel100.json > /dev/null || exit 1
      echo "pmc4 done"; grep -E "hbm_bytes_per_search|avg_launch|k_scan" $O/pmc_config4_sel100.json ;;
    index)
      bash tools/gpu_index_pmc.sh 2:nprobe=1 3:nprobe=1 > $O/index_pmc.log 2>&1 || { echo "index pmc failed"; tail -20 $O/index_pmc.log; exit 1; }
      cp gpurun_out/index_pmc.json $O/index_pmc.json && grep -E "hbm_bytes_per_search|search" $O/index_pmc.json | head -8 ;;
    risk)
      timeout -k 10 600 python -u tools/blas_order_risk.py --out $O/blas_order_risk.json > $O/blas_order_risk.log 2>&1 \
        || { echo "risk failed"; tail -20 $O/blas_order_risk.log; exit 1; }
      grep -A4 per_block $O/blas_order_risk.json ;;
    bench)
      # this session's PMC summaries when it made them, else the committed ones
      PA=()
      [ -f $O/pmc_traffic.json ] && PA+=(--pmc $O/pmc_traffic.json)
      [ -f $O/pmc_nq1.json ] && PA+=(--pmc-nq1 $O/pmc_nq1.json)
      [ -f $O/index_pmc.json ] && PA+=(--index-pmc $O/index_pmc.json)
      timeout -k 10 900 python -u bench.py "${PA[@]}" \
        > $O/bench.json 2> $O/bench.err || { echo "bench failed rc=$?"; tail -30 $O/bench.err; exit 1; }
      head -c 3000 $O/bench.json; echo
      ( cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prof" -o run --output-format csv \
          -- python "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --no-cpu --no-verify --no-index --no-configs \
          --no-config1-points > "$GRAFT_REPO_ROOT/$O/prof_bench.json" 2> "$GRAFT_REPO_ROOT/$O/prof.err" ) \
        || { echo "rocprof failed"; tail -20 $O/prof.err; exit 1; }
      python tools/pp_per_search.py $O/prof/run_kernel_trace.csv > $O/bench_p4m_per_search.txt && tail -4 $O/bench_p4m_per_search.txt
      echo "rocprof done" ;;
  esac
done
