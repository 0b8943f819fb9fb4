#!/bin/bash
# Index list-count sweep at BASELINE configs[2] size (10M x 768 cosine, nq 1000,
# k 100): for each "mode:nlist" pair one build, then an nprobe sweep.  Each
# build + sweep has its own time limit; the first failure ends the session.
#   bash tools/gpu_index_nlist.sh "3:65536 3:32768 2:65536" "nprobe=1;nprobe=2;..."
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/nlist
PAIRS="$1"
SEARCH="${2:-nprobe=1;nprobe=2;nprobe=4;nprobe=8;nprobe=16;nprobe=32;nprobe=64}"
for pr in $PAIRS; do
  mode=${pr%%:*}; nl=${pr##*:}
  out=gpurun_out/nlist/m${mode}_nl${nl}
  timeout -k 10 400 python -u tools/index_sweep.py --mode "$mode" --build "nlist=$nl" --search "$SEARCH" --reps 3 \
      > $out.jsonl 2> $out.err
  rc=$?; echo "mode $mode nlist $nl rc=$rc"; cut -c1-420 $out.jsonl; tail -3 $out.err
  [ $rc -ne 0 ] && exit 1
done
exit 0
