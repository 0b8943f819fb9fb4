#!/bin/bash
# Ingest kernel times: rocprofv3 kernel-trace stats of tools/ingest_bench.py
# (quantised 1M x 768).  Output under gpurun_out/ingest_prof/.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/ingest_prof
mkdir -p $O
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O -o run --output-format csv \
    -- python3 $GRAFT_REPO_ROOT/tools/ingest_bench.py --kind quantised --reps 1 > $O/bench.out 2> $O/bench.err ) \
  || { echo "rocprof failed"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.out
f=$(find $O -name "*kernel_stats.csv" | head -1); cut -c1-220 "$f" | head -20
