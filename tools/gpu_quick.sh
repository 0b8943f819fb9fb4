#!/bin/bash
# tests + nq sweep (no bench)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/gpu_tests.log
[ $rc -ne 0 ] && exit 1
timeout -k 10 400 python tools/sweep.py "$@" > gpurun_out/sweep.jsonl 2> gpurun_out/sweep.err
echo "sweep rc=$?"; cat gpurun_out/sweep.jsonl; tail -5 gpurun_out/sweep.err
