#!/bin/bash
# index tests + 10M sweep + kernel trace of the sweep
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_index.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/gpu_index_tests.log 2>&1
rc=$?; echo "index tests rc=$rc"; tail -3 gpurun_out/gpu_index_tests.log
[ $rc -ne 0 ] && exit 1
timeout -k 10 300 python -u tools/index_sweep.py --search "nprobe=2;nprobe=4;nprobe=8" "$@" > gpurun_out/isw.jsonl 2> gpurun_out/isw.err
rc=$?; echo "sweep rc=$rc"; cut -c1-420 gpurun_out/isw.jsonl
[ $rc -ne 0 ] && exit 1
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/iprofq" -o run --output-format csv \
    -- python "$GRAFT_REPO_ROOT/tools/index_sweep.py" --reps 2 --search "nprobe=2" > /dev/null 2> "$GRAFT_REPO_ROOT/gpurun_out/iprofq.err" )
echo "rocprof rc=$?"
