#!/bin/bash
# same-box A/B of two builds of libmqvs.so (ab/libmqvs_old.so, ab/libmqvs_new.so)
# on the headline batch: new, old, new, old.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
for arm in new old new old; do
  cp ab/libmqvs_$arm.so myscaledb_amd/libmqvs.so || exit 1
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-index --no-configs --no-config1-points \
    --no-cpu --no-small --no-verify --read-sweep-gib 0 > gpurun_out/ab_$arm.json 2> gpurun_out/ab_$arm.err || { echo "$arm failed"; tail -5 gpurun_out/ab_$arm.err; exit 1; }
  python3 -c "
import json; d = json.loads(open('gpurun_out/ab_$arm.json').read().strip().splitlines()[-1]); st = d['stats_last_step']
print('$arm', d['value'], d['ms_per_step'], st['main_ms'], st['probe_ms'], st['final_ms'])"
done
cp ab/libmqvs_new.so myscaledb_amd/libmqvs.so
