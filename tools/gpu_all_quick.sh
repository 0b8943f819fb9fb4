#!/bin/bash
# all GPU tests, binary sweep, quick flat bench (no CPU baseline / index leg)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/gpu_tests.log
[ $rc -ne 0 ] && exit 1
timeout -k 10 300 python -u tools/binary_sweep.py > gpurun_out/binary_sweep.jsonl 2> gpurun_out/binary_sweep.err
echo "sweep rc=$?"; cut -c1-330 gpurun_out/binary_sweep.jsonl
[ "$1" = "--no-bench" ] && exit 0
timeout -k 10 300 python -u bench.py --no-cpu --no-verify "$@" > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err
echo "bench rc=$?"; python -c "
import json; r=json.load(open('gpurun_out/bench_quick.json')); print(r['value'], r['ms_per_step'], r['stats_last_step']); print(r.get('index',{}).get('points'))"
