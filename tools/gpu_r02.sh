#!/bin/bash
# One GPU session (round 2): GPU tests, bench line, rocprof kernel-trace
# summary of the same bench, PMC passes of the batch search.  Every GPU step
# has its own time limit; the first failure ends the session.
#   bash tools/gpu_r02.sh [--no-tests] [--no-pmc] [-- extra bench args]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TESTS=1; PMC=1
while [ $# -gt 0 ]; do
  case "$1" in
    --no-tests) TESTS=0; shift ;;
    --no-pmc) PMC=0; shift ;;
    --) shift; break ;;
    *) break ;;
  esac
done
if [ $TESTS = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/gpu_tests.log
  [ $rc -ne 0 ] && exit 1
fi
timeout -k 10 600 python -u bench.py "$@" > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed rc=$?"; tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
( cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run --output-format csv \
    -- python "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --no-cpu --no-verify --no-small --no-index --no-configs "$@" \
    > "$GRAFT_REPO_ROOT/gpurun_out/prof_bench.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/prof.err" )
rc=$?; echo "rocprof rc=$rc"; [ $rc -ne 0 ] && exit 1
[ $PMC = 0 ] && exit 0
bash tools/gpu_pmc.sh python bench.py --steps 2 --warmup 0 --no-cpu --no-verify --no-index --no-small --no-configs "$@" || exit 1
python tools/pmc_traffic.py gpurun_out --searches 2 --nq 1000 --out gpurun_out/pmc_traffic.json > /dev/null
echo "pmc summary rc=$?"
