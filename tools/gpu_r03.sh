#!/bin/bash
# One GPU session (round 3): selected GPU tests, then an A/B of the batch
# scan (tools/ab_split.py args after --).  Each GPU step has its own time
# limit; the first failure ends the session.
#   bash tools/gpu_r03.sh "<pytest targets>" [-- ab args]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TARGETS="$1"; shift
if [ -n "$TARGETS" ] && [ "$TARGETS" != "none" ]; then
  timeout -k 10 900 python -u -m pytest $TARGETS -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/gpu_tests.log | tail -5
  [ $rc -ne 0 ] && { grep -B5 -A40 "FAILED\|Error" gpurun_out/gpu_tests.log | head -80; exit 1; }
fi
[ "$1" = "--" ] || exit 0
shift
timeout -k 10 600 python -u tools/ab_split.py "$@" > gpurun_out/ab.jsonl 2> gpurun_out/ab.err
rc=$?; echo "ab rc=$rc"; cat gpurun_out/ab.jsonl; tail -5 gpurun_out/ab.err
exit $rc
