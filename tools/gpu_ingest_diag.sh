#!/bin/bash
# Decode-time decomposition of the LZ4 ingest (measurement library, wrong
# output in the DIAG variants): tools/ingest_bench.py quantised per variant.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ingest_diag
for dg in ${DIAGS:-0 1}; do
  timeout -k 10 120 env MQVS_LZ4_DIAG=$dg python3 -u tools/ingest_bench.py --dbg --kind quantised --reps 2 \
      > gpurun_out/ingest_diag/d$dg.out 2> gpurun_out/ingest_diag/d$dg.err || { echo "diag $dg failed"; tail -5 gpurun_out/ingest_diag/d$dg.err; exit 1; }
  echo "diag $dg: $(cut -c1-400 gpurun_out/ingest_diag/d$dg.out)"
done
