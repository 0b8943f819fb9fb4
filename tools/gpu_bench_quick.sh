#!/bin/bash
# bench.py only (extra args passed through), output to gpurun_out/bench_quick.json
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py "$@" > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench_quick.err; exit $rc
