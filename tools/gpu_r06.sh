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
    cpu)
      timeout -k 10 600 python -u tools/host_cpu_wait.py > $O/host_cpu_wait.jsonl 2> $O/host_cpu_wait.err \
        || { echo "cpu wait failed"; tail -20 $O/host_cpu_wait.err; exit 1; }
      cat $O/host_cpu_wait.jsonl ;;
  esac
done
