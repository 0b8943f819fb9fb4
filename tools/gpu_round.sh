#!/bin/bash
# One GPU session: tests, bench, rocprof kernel-trace summary, PMC traffic.
# Each GPU step has its own time limit; the first failure ends the session.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/gpu_tests.log
[ $rc -ne 0 ] && exit 1
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed rc=$?"; tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
( cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run --output-format csv \
    -- python "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --no-cpu --no-verify \
    > "$GRAFT_REPO_ROOT/gpurun_out/prof_bench.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/prof.err" )
rc=$?; echo "rocprof rc=$rc"; [ $rc -ne 0 ] && exit 1
[ "$1" = "--no-pmc" ] && exit 0
bash tools/gpu_pmc.sh python bench.py --steps 2 --warmup 0 --no-cpu --no-verify --no-index || exit 1
python tools/pmc_traffic.py gpurun_out --searches 2 --out gpurun_out/pmc_traffic.json > /dev/null
echo "pmc summary rc=$?"
