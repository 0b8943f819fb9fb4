#!/bin/bash
# GPU tests (optionally a -m expression), then an A/B (tools/ab_split.py args after --)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
M="${1:-gpu and not fullsize}"; shift
timeout -k 10 900 python -u -m pytest tests -m "$M" -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/gpu_tests.log
[ $rc -ne 0 ] && exit 1
[ "$1" = "--" ] || exit 0
shift
timeout -k 10 900 python -u tools/ab_split.py "$@" > gpurun_out/ab.jsonl 2> gpurun_out/ab.err
rc=$?; echo "ab rc=$rc"; cut -c1-330 gpurun_out/ab.jsonl; tail -3 gpurun_out/ab.err
exit $rc
