#!/bin/bash
# small-nq fixed-cost A/B: main-scan segmentation / probe target (MQVS_SEG)
# at nq 1/4/16 on 10M x 768 cosine, then a rocprofv3 kernel trace of nq 1
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/segab
TUNES="${1:-;MQVS_SEG=8,4,65536;MQVS_SEG=8,4,32768;MQVS_SEG=16,4,65536;MQVS_SEG=4,8,65536;MQVS_SEG=16,8,131072}"
timeout -k 10 400 python -u tools/ab_split.py --nqs "${2:-1,4,16}" --splits 2 --reps 20 --tunes "$TUNES" \
    > gpurun_out/segab/ab.jsonl 2> gpurun_out/segab/ab.err
rc=$?; echo "ab rc=$rc"; cut -c1-700 gpurun_out/segab/ab.jsonl; tail -3 gpurun_out/segab/ab.err
[ $rc -ne 0 ] && exit 1
[ "$3" = "--prof" ] || exit 0
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/segab/prof -o run -- python -u tools/ab_split.py --nqs 1 --splits 2 --reps 20 --no-exact > gpurun_out/segab/prof.log 2>&1
rc=$?; echo "prof rc=$rc"
f=$(find gpurun_out/segab/prof -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cut -c1-160 "$f" | head -30
exit $rc
