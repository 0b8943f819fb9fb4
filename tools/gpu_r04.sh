#!/bin/bash
# round-4 GPU check: the GPU test suite, then a short headline bench
# (configs[1] only).  usage: tools/gpu_r04.sh [tests|bench|all] [bench args...]
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
what=${1:-all}
shift
if [ "$what" = tests ] || [ "$what" = all ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/gpu_tests.log 2>&1
  rc=$?
  echo "pytest rc=$rc"; tail -5 gpurun_out/gpu_tests.log
  [ $rc -ne 0 ] && exit 1
fi
if [ "$what" = bench ] || [ "$what" = all ]; then
  timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-index --no-configs --no-config1-points \
    --no-cpu --no-small --read-sweep-gib 0 "$@" > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err
  rc=$?
  echo "bench rc=$rc"; tail -3 gpurun_out/bench_quick.err
  python3 - <<'EOF'
import json
d = json.loads(open("gpurun_out/bench_quick.json").read().strip().splitlines()[-1])
st = d["stats_last_step"]
print(json.dumps({"value": d["value"], "ms": d["ms_per_step"], "exact": d["exact_check"],
                  "frac": d["roofline"]["frac"], "main_ms": st["main_ms"], "probe_ms": st["probe_ms"],
                  "probe_select_ms": st["probe_select_ms"], "refine_ms": st["refine_ms"], "final_ms": st["final_ms"],
                  "segments": st["segments"], "rescans": st["rescans"], "survivors_max": st["survivors_max"],
                  "candidates_max": st["candidates_max"]}))
EOF
  [ $rc -ne 0 ] && exit 1
fi
exit 0
