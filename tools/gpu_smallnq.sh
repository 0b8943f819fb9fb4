#!/bin/bash
# small-batch breakdown: per-search stats (sweep.py) + rocprof kernel stats
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/smallnq
NQS="${1:-1,4,16,64}"
timeout -k 10 300 python -u tools/sweep.py --nqs "$NQS" --metrics Cosine --reps 5 > gpurun_out/smallnq/sweep.jsonl 2> gpurun_out/smallnq/sweep.err
rc=$?; echo "sweep rc=$rc"; cut -c1-900 gpurun_out/smallnq/sweep.jsonl; tail -3 gpurun_out/smallnq/sweep.err
[ $rc -ne 0 ] && exit 1
[ "$2" = "--prof" ] || exit 0
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/smallnq/prof -o run -- python -u tools/sweep.py --nqs 1 --metrics Cosine --reps 20 > gpurun_out/smallnq/prof.log 2>&1
rc=$?; echo "prof rc=$rc"
f=$(find gpurun_out/smallnq/prof -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cut -c1-200 "$f" | head -30
exit $rc
