#!/bin/bash
# GPU tests (fast suite) then a pre-filter A/B (tools/ab_split.py args after --)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "$1" != "--no-tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/gpu_tests.log
  [ $rc -ne 0 ] && exit 1
else
  shift
fi
[ "$1" = "--" ] && shift
timeout -k 10 900 python -u tools/ab_split.py "$@" > gpurun_out/ab.jsonl 2> gpurun_out/ab.err
rc=$?; echo "ab rc=$rc"; cat gpurun_out/ab.jsonl; tail -5 gpurun_out/ab.err
exit $rc
