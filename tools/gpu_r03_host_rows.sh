#!/bin/bash
# Host-resident rows: their GPU tests (+ shim), then the timing on the bench part.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r03c
timeout -k 10 300 python -u -m pytest tests/test_gpu_host_rows.py tests/test_shim.py tests/test_abi.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r03c/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASSED|FAILED|Error|passed|failed" gpurun_out/r03c/tests.log | tail -12
[ $rc -ne 0 ] && { grep -A30 "FAILED\|Error" gpurun_out/r03c/tests.log | head -60; exit 1; }
timeout -k 10 300 python -u tools/host_rows_bench.py > gpurun_out/r03c/host_rows.jsonl 2> gpurun_out/r03c/host_rows.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/r03c/host_rows.jsonl; tail -3 gpurun_out/r03c/host_rows.err
exit $rc
