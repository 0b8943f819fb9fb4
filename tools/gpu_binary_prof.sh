#!/bin/bash
# binary tests, sweep, and a kernel trace of the sweep
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_binary.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_binary_tests.log 2>&1
rc=$?; echo "binary pytest rc=$rc"; tail -3 gpurun_out/gpu_binary_tests.log
[ $rc -ne 0 ] && exit 1
timeout -k 10 300 python -u tools/binary_sweep.py "$@" > gpurun_out/binary_sweep.jsonl 2> gpurun_out/binary_sweep.err
echo "sweep rc=$?"; cut -c1-260 gpurun_out/binary_sweep.jsonl
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/bprof" -o run --output-format csv \
    -- python "$GRAFT_REPO_ROOT/tools/binary_sweep.py" --reps 2 "$@" > /dev/null 2> "$GRAFT_REPO_ROOT/gpurun_out/bprof.err" )
echo "rocprof rc=$?"
