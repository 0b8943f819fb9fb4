#!/bin/bash
# plane-layout check: the GPU suite, then the headline batch (configs[1]) and
# the configs[3]/[4] legs.  Outputs gpurun_out/r04_layout/.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04_layout
mkdir -p $O
if [ "${1:-tests}" = tests ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 $O/gpu_tests.log; [ $rc -ne 0 ] && exit 1
fi
timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 --no-index --no-config1-points --no-cpu --no-small \
  --read-sweep-gib 0 --no-verify > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/r04_layout/bench.json").read().strip().splitlines()[-1])
st = d["stats_last_step"]
print(json.dumps({"value": d["value"], "ms": d["ms_per_step"], "main_ms": st["main_ms"], "frac": d["roofline"]["frac"]}))
for name, c in d.get("configs", {}).items():
    for p in c.get("points", []):
        print(name, {k: p.get(k) for k in ("nq", "selectivity_pct", "ms_per_search", "main_ms", "plane_bytes_read", "end_to_end_gbs")}, p["exact"]["ids_equal"] and p["exact"]["dist_bitwise_equal"])
PY
