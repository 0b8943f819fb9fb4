#!/bin/bash
# Index path on the GPU: its tests, then sweeps (1M, then BASELINE configs[2] 10M x 768).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_index.py -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/gpu_index_tests.log 2>&1
rc=$?; echo "index tests rc=$rc"; tail -25 gpurun_out/gpu_index_tests.log
[ $rc -ne 0 ] && exit 1
timeout -k 10 200 python -u tools/index_sweep.py --n 1000000 "$@" > gpurun_out/index_sweep_1m.jsonl 2> gpurun_out/index_sweep_1m.err
rc=$?; echo "sweep 1M rc=$rc"; cat gpurun_out/index_sweep_1m.jsonl; tail -5 gpurun_out/index_sweep_1m.err
[ $rc -ne 0 ] && exit 1
timeout -k 10 400 python -u tools/index_sweep.py "$@" > gpurun_out/index_sweep_10m.jsonl 2> gpurun_out/index_sweep_10m.err
rc=$?; echo "sweep 10M rc=$rc"; cat gpurun_out/index_sweep_10m.jsonl; tail -5 gpurun_out/index_sweep_10m.err
