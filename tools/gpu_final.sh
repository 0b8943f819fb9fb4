#!/bin/bash
# smoke + bench (N=1) + rocprof kernel-trace summary of the same bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 500 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed rc=$?"; tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
( cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run --output-format csv \
    -- python "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --no-cpu --no-verify \
    > "$GRAFT_REPO_ROOT/gpurun_out/prof_bench.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/prof.err" )
echo "rocprof rc=$?"
