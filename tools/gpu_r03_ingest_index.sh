#!/bin/bash
# Round-3 session: the grouped LZ4 decoder (ingest tests + rate) and the
# index at 65536 lists (tests, then list-count / coarse-stage sweeps on the
# measurement library).  Each GPU step has its own time limit; the first
# failure ends the session.  Outputs under gpurun_out/r03b/.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03b
mkdir -p $O
run() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "== $name rc=$rc"; tail -c 2500 $O/$name.out
  [ $rc -ne 0 ] && { tail -30 $O/$name.err; exit 1; }
  return 0
}
STEPS="${*:-ingest index sweep}"
for step in $STEPS; do
  case $step in
    ingest)
      run ingest_tests 300 python -u -m pytest tests/test_gpu_ingest.py -m gpu -x -q --timeout 120 --timeout-method thread
      run ingest_bench 300 python -u tools/ingest_bench.py ;;
    index)
      run index_tests 300 python -u -m pytest tests/test_gpu_index.py tests/test_gpu_cache.py tests/test_shim.py -m gpu -x -q --timeout 120 --timeout-method thread ;;
    dflt)
      S="nprobe=1;nprobe=2;nprobe=4;nprobe=8;nprobe=16;nprobe=32;alpha=3"
      run m3_dflt 300 python -u tools/index_sweep.py --mode 3 --search "$S" --reps 3
      run m2_dflt 300 python -u tools/index_sweep.py --mode 2 --search "$S" --reps 3
      run m3_16384 300 python -u tools/index_sweep.py --mode 3 --build nlist=16384 --search "nprobe=4;nprobe=8;nprobe=16;nprobe=32;nprobe=64" --reps 3 ;;
    sweep)
      S="nprobe=1;nprobe=2;nprobe=4;nprobe=8;nprobe=16;nprobe=32"
      run m3_65536_flat 300 env MQVS_IVF_COARSE=1 python -u tools/index_sweep.py --dbg --mode 3 --build nlist=65536 --search "$S" --reps 3
      run m3_65536_list 300 env MQVS_IVF_COARSE=0 python -u tools/index_sweep.py --dbg --mode 3 --build nlist=65536 --search "nprobe=1;nprobe=2" --reps 3
      run m2_65536 300 python -u tools/index_sweep.py --dbg --mode 2 --build nlist=65536 --search "$S" --reps 3
      run m2_16384 300 python -u tools/index_sweep.py --dbg --mode 2 --build nlist=16384 --search "$S" --reps 3
      run m3_65536_s1m 300 python -u tools/index_sweep.py --dbg --mode 3 --build nlist=65536,sample=1048576 --search "nprobe=1;nprobe=2;nprobe=4" --reps 3
      run m2_10000_flat 300 python -u tools/index_sweep.py --dbg --mode 2 --build nlist=10000 --search "nprobe=2;nprobe=4;nprobe=8" --reps 3 ;;
  esac
done
exit 0
