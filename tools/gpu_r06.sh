#!/bin/bash
# Round-6 GPU session steps (each GPU step under its own time limit; the
# first failure ends the session).  Outputs under gpurun_out/r06/.
#   bash tools/gpu_r06.sh [tests|idx|cpu|alltests]...
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06
mkdir -p $O
for step in "$@"; do
  case $step in
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
    lds)
      bash tools/gpu_lds_pmc.sh 0 8 4 6 || exit 1 ;;
    cpu)
      timeout -k 10 600 python -u tools/host_cpu_wait.py > $O/host_cpu_wait.jsonl 2> $O/host_cpu_wait.err \
        || { echo "cpu wait failed"; tail -20 $O/host_cpu_wait.err; exit 1; }
      cat $O/host_cpu_wait.jsonl ;;
  esac
done
