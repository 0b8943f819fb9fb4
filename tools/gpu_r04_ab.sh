#!/bin/bash
# A/B of batch-kernel variants (measurement build) at configs[1]: one process,
# arms interleaved.  usage: tools/gpu_r04_ab.sh 'ENV=V;ENV=V;...' [metrics]
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/ab_split.py --dbg --nqs 1000 --metrics "${2:-Cosine}" --modes 1 --splits 2 --reps 5 \
  --tunes "$1" > gpurun_out/ab.jsonl 2> gpurun_out/ab.err
rc=$?
tail -2 gpurun_out/ab.err
python3 -c "
import json
for l in open('gpurun_out/ab.jsonl'):
    d=json.loads(l); print(d['tune'], d['metric'], 'main', d['main_ms'], 'wall', d['wall_ms'], 'eq', d['bitwise_eq_exact'])
"
exit $rc
