#!/bin/bash
# binary scan: grid-size sweep at small nq + kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/bin_tune.jsonl
for g in 1024 2048 4096 8192 16384 65536; do
  MQVS_BIN_GRID=$g timeout -k 10 120 python -u tools/binary_sweep.py --nq 1,8,1000 --metric Hamming --reps 4 > gpurun_out/bt.jsonl 2>>gpurun_out/bin_tune.err || exit 1
  sed "s/^{/{\"grid\": $g, /" gpurun_out/bt.jsonl >> gpurun_out/bin_tune.jsonl
done
cut -c1-200 gpurun_out/bin_tune.jsonl
( cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/bprof2" -o run --output-format csv \
    -- python "$GRAFT_REPO_ROOT/tools/binary_sweep.py" --reps 2 --nq 1 --metric Hamming > /dev/null 2> "$GRAFT_REPO_ROOT/gpurun_out/bprof2.err" )
echo "rocprof rc=$?"
