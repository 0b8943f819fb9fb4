#!/bin/bash
# binary-vector GPU tests + scan sweep
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_binary.py -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_binary_tests.log 2>&1
rc=$?; echo "binary pytest rc=$rc"; tail -15 gpurun_out/gpu_binary_tests.log
[ $rc -ne 0 ] && exit 1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "all gpu pytest rc=$rc"; tail -4 gpurun_out/gpu_tests.log
[ $rc -ne 0 ] && exit 1
timeout -k 10 300 python -u tools/binary_sweep.py "$@" > gpurun_out/binary_sweep.jsonl 2> gpurun_out/binary_sweep.err
echo "sweep rc=$?"; cat gpurun_out/binary_sweep.jsonl | cut -c1-300; tail -3 gpurun_out/binary_sweep.err
