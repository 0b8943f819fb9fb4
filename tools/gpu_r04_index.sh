#!/bin/bash
# round-4 index check: configs[2] sweeps on both distributions, the default
# coarse step (batch-kernel group maxima + pick) against the FLAT coarse
# search (measurement build, MQVS_IVF_COARSE=1).  Outputs gpurun_out/r04_index/.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04_index
mkdir -p $O
run() {  # tag, seconds, command...
  local tag=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > $O/$tag.jsonl 2> $O/$tag.err || { echo "$tag failed rc=$?"; tail -20 $O/$tag.err; exit 1; }
  echo "== $tag"; cut -c1-330 $O/$tag.jsonl
}
run m3 300 python -u tools/index_sweep.py --mode 3 --search "nprobe=1;nprobe=2;nprobe=4" --reps 5
run m2 300 python -u tools/index_sweep.py --mode 2 --search "nprobe=1;nprobe=2;nprobe=4;nprobe=8" --reps 5
if [ "${1:-}" = ab ]; then
  run m3_flat 300 env MQVS_IVF_COARSE=1 python -u tools/index_sweep.py --dbg --mode 3 --search "nprobe=1;nprobe=2" --reps 5
fi
exit 0
