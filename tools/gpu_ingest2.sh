#!/bin/bash
# full GPU suite, then column-ingest bench (with / without block checksums) + kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/gpu_tests.log
[ $rc -ne 0 ] && exit 1
timeout -k 10 400 python -u tools/ingest_bench.py > gpurun_out/ingest_bench.jsonl 2> gpurun_out/ingest_bench.err || { echo "bench failed"; tail -5 gpurun_out/ingest_bench.err; exit 1; }
cat gpurun_out/ingest_bench.jsonl
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/iprof_ing" -o run --output-format csv \
    -- python "$GRAFT_REPO_ROOT/tools/ingest_bench.py" --reps 1 > /dev/null 2> "$GRAFT_REPO_ROOT/gpurun_out/iprof_ing.err" )
echo "rocprof rc=$?"
