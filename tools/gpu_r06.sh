#!/bin/bash
# Round-6 GPU session steps (each GPU step under its own time limit; the
# first failure ends the session).  Outputs under gpurun_out/r06/.
#   bash tools/gpu_r06.sh [tests|idx|cpu|alltests]...
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06
mkdir -p $O
pmc_set() {  # tag, searches, args...
  local tag=$1 s=$2; shift 2
  bash tools/gpu_pmc.sh python tools/pmc_search.py --searches "$s" "$@" || return 1
  rm -rf "$O/pmc_$tag" && mkdir -p "$O/pmc_$tag" && mv gpurun_out/pmc1 gpurun_out/pmc2 gpurun_out/pmc3 gpurun_out/pmc*.log "$O/pmc_$tag/" || return 1
}
for step in "$@"; do
  case $step in
    pmc)
      pmc_set config1 2 --nq 1000 || exit 1
      python tools/pmc_traffic.py $O/pmc_config1 --searches 3 --nq 1000 --out $O/pmc_traffic.json > /dev/null || exit 1
      pmc_set nq1 4 --nq 1 || exit 1
      python tools/pmc_traffic.py $O/pmc_nq1 --searches 5 --nq 1 --out $O/pmc_nq1.json > /dev/null || exit 1
      echo "pmc done"; cat $O/pmc_traffic.json $O/pmc_nq1.json | grep -E "hbm_bytes_per_search|avg_launch|clock|mfma_busy|k_scan" ;;
    pmc4)
      for sel in 10 1; do
        pmc_set config4_sel$sel 4 --nq 1 --n 50000000 --metric L2 --selectivity $sel || exit 1
        python tools/pmc_traffic.py $O/pmc_config4_sel$sel --searches 5 --nq 1 --out $O/pmc_config4_sel$sel.json > /dev/null || exit 1
        rm -rf $O/pmc_config4_sel$sel/pmc1 $O/pmc_config4_sel$sel/pmc2 $O/pmc_config4_sel$sel/pmc3
        grep -E "hbm_bytes_per_search|avg_launch" $O/pmc_config4_sel$sel.json
      done ;;
    index)
      bash tools/gpu_index_pmc.sh 2:nprobe=1 3:nprobe=1 > $O/index_pmc.log 2>&1 || { echo "index pmc failed"; tail -20 $O/index_pmc.log; exit 1; }
      cp gpurun_out/index_pmc.json $O/index_pmc.json && grep -E "hbm_bytes_per_search|search" $O/index_pmc.json | head -8 ;;
    ingest)
      timeout -k 10 400 python -u tools/ingest_bench.py > $O/ingest_bench_1Mx768.jsonl 2> $O/ingest_bench.err \
        || { echo "ingest failed"; tail -5 $O/ingest_bench.err; exit 1; }
      cat $O/ingest_bench_1Mx768.jsonl | cut -c1-300 ;;
    tl)  # kernel timelines: nq 1 and configs[4] 1 %
      for t in nq1 sel1; do
        a="--nq 1 --searches 4"; st=k_query_prep
        [ $t = sel1 ] && a="--nq 1 --n 50000000 --metric L2 --selectivity 1 --searches 4" && st=k_chunk_count
        ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/tr_$t" -o run --output-format csv \
            -- python3 "$GRAFT_REPO_ROOT/tools/pmc_search.py" $a > "$GRAFT_REPO_ROOT/$O/tr_$t.log" 2>&1 ) || { echo "trace $t failed"; exit 1; }
        python3 tools/timeline.py $O/tr_$t/run_kernel_trace.csv --start $st --nth -1 | tee $O/${t}_timeline.txt
      done ;;
    bench)
      PA=()
      [ -f $O/pmc_traffic.json ] && PA+=(--pmc $O/pmc_traffic.json)
      [ -f $O/pmc_nq1.json ] && PA+=(--pmc-nq1 $O/pmc_nq1.json)
      [ -f $O/index_pmc.json ] && PA+=(--index-pmc $O/index_pmc.json)
      timeout -k 10 900 python -u bench.py "${PA[@]}" > $O/bench.json 2> $O/bench.err || { echo "bench failed rc=$?"; tail -30 $O/bench.err; exit 1; }
      head -c 3000 $O/bench.json; echo
      ( cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prof" -o run --output-format csv \
          -- python "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --no-cpu --no-verify --no-index --no-configs \
          --no-config1-points > "$GRAFT_REPO_ROOT/$O/prof_bench.json" 2> "$GRAFT_REPO_ROOT/$O/prof.err" ) \
        || { echo "rocprof failed"; tail -20 $O/prof.err; exit 1; }
      python tools/pp_per_search.py $O/prof/run_kernel_trace.csv > $O/bench_p4m_per_search.txt && tail -4 $O/bench_p4m_per_search.txt
      echo "rocprof done" ;;
    tests)
      timeout -k 10 900 python -u -m pytest tests/test_gpu_index.py tests/test_gpu_concurrency.py tests/test_gpu_rccl_world1.py tests/test_gpu_sharded.py tests/test_gpu_bench_loopback.py -x -v \
        --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
      tail -3 $O/tests.log ;;
    alltests)
      timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
        > $O/alltests.log 2>&1 || { echo "alltests failed"; tail -40 $O/alltests.log; exit 1; }
      tail -3 $O/alltests.log ;;
    idx)
      for m in 3 2; do
        for ra in "" "--rerank-all"; do
          timeout -k 10 300 python -u tools/index_sweep.py --mode $m --search "nprobe=1;nprobe=2" --reps 5 $ra \
            >> $O/isweep.jsonl 2>> $O/isweep.err || { echo "sweep failed"; tail -20 $O/isweep.err; exit 1; }
        done
      done
      cut -c1-600 $O/isweep.jsonl ;;
    ab)
      timeout -k 10 600 python -u tools/ab_split.py --dbg --nqs 1000 --splits 2 --modes 1 --metrics Cosine,L2 \
        --tunes 'MQVS_P4M_DIAG=0;MQVS_P4M_DIAG=8;MQVS_P4M_DIAG=0;MQVS_P4M_DIAG=8' --reps 5 \
        > $O/ab_walk.jsonl 2> $O/ab_walk.err || { echo "ab failed"; tail -20 $O/ab_walk.err; exit 1; }
      cut -c1-400 $O/ab_walk.jsonl ;;
    rr)
      # index A/B arms of the measurement build: IDX_ARMS="ENV=V,ENV=V;..." ('-' = defaults)
      IFS=';' read -ra ARMS <<< "${IDX_ARMS:--;MQVS_IVF_PAIR=0}"
      for arm in "${ARMS[@]}"; do
        ( [ "$arm" != "-" ] && for kv in ${arm//,/ }; do export "$kv"; done
          timeout -k 10 300 python -u tools/index_sweep.py --dbg --mode ${IDX_MODE:-3} --search "${IDX_SEARCH:-nprobe=1}" --reps 7 \
            | sed "s/^{/{\"arm\": \"$arm\", /" ) >> $O/rr_ab.jsonl 2>> $O/rr_ab.err || { echo "rr failed"; tail -20 $O/rr_ab.err; exit 1; }
      done
      grep search $O/rr_ab.jsonl | cut -c1-460 ;;
    itl)
      # kernel timeline of one mode-3 nprobe=1 index search (k_to_bf16 opens a search)
      ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/$O/itl" -o run \
          -- python "$GRAFT_REPO_ROOT/tools/index_search_run.py" --mode 3 --search nprobe=1 --searches 3 \
          > "$GRAFT_REPO_ROOT/$O/itl.log" 2>&1 ) || { echo "itl failed"; tail -5 $O/itl.log; exit 1; }
      python3 tools/timeline.py $O/itl/run_kernel_trace.csv --start k_to_bf16 --nth -1 | tee $O/index_m3_nprobe1_timeline.txt ;;
    api)
      # kernel + host HIP-call timelines: one mode-3 nprobe=1 index search, one nq 1 FLAT search
      ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d "$GRAFT_REPO_ROOT/$O/api_idx" -o run \
          -- python "$GRAFT_REPO_ROOT/tools/index_search_run.py" --mode 3 --search nprobe=1 --searches 3 \
          > "$GRAFT_REPO_ROOT/$O/api_idx.log" 2>&1 ) || { echo "api idx failed"; tail -5 $O/api_idx.log; exit 1; }
      python3 tools/timeline.py $O/api_idx/run_kernel_trace.csv --api $O/api_idx/run_hip_api_trace.csv --start k_to_bf16 --nth -1 > $O/api_idx.txt
      ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d "$GRAFT_REPO_ROOT/$O/api_nq1" -o run \
          -- python3 "$GRAFT_REPO_ROOT/tools/pmc_search.py" --nq 1 --searches 4 > "$GRAFT_REPO_ROOT/$O/api_nq1.log" 2>&1 ) \
        || { echo "api nq1 failed"; tail -5 $O/api_nq1.log; exit 1; }
      python3 tools/timeline.py $O/api_nq1/run_kernel_trace.csv --api $O/api_nq1/run_hip_api_trace.csv --start k_query_prep --nth -1 > $O/api_nq1.txt
      head -30 $O/api_idx.txt ;;
    wab)
      timeout -k 10 400 python -u tools/wait_ab.py > $O/wait_ab.jsonl 2> $O/wait_ab.err \
        || { echo "wait ab failed"; tail -20 $O/wait_ab.err; exit 1; }
      cat $O/wait_ab.jsonl ;;
    seg)
      # nq 1 segmentation A/B (measurement build): SEG_TUNES="MQVS_SEG=a,b,c;..."
      timeout -k 10 600 python -u tools/ab_split.py --dbg --nqs 1 --splits 2 --modes 1 --metrics Cosine \
        --tunes "${SEG_TUNES:-MQVS_SEG=8,4,65536;MQVS_SEG=32,4,65536}" --reps 15 \
        > $O/seg_ab.jsonl 2> $O/seg_ab.err || { echo "seg ab failed"; tail -20 $O/seg_ab.err; exit 1; }
      cut -c1-400 $O/seg_ab.jsonl ;;
    lds)
      bash tools/gpu_lds_pmc.sh 0 8 4 6 || exit 1 ;;
    cpu)
      timeout -k 10 600 python -u tools/host_cpu_wait.py > $O/host_cpu_wait.jsonl 2> $O/host_cpu_wait.err \
        || { echo "cpu wait failed"; tail -20 $O/host_cpu_wait.err; exit 1; }
      cat $O/host_cpu_wait.jsonl ;;
  esac
done
