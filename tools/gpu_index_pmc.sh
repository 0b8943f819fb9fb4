#!/bin/bash
# PMC passes of the index scan (k_ivf_scan) at given operating points:
#   bash tools/gpu_index_pmc.sh 2:nprobe=2 3:nprobe=512
# -> gpurun_out/index_pmc.json  {mode: pmc_traffic.py summary + "search"}
set -o pipefail
R="$GRAFT_REPO_ROOT"
cd "$R" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/index_pmc
for spec in "$@"; do
    mode=${spec%%:*}; search=${spec#*:}
    rm -rf gpurun_out/pmc1 gpurun_out/pmc2 gpurun_out/pmc3
    bash tools/gpu_pmc.sh python tools/index_search_run.py --mode "$mode" --search "$search" --searches 2 \
        --info-out "$R/gpurun_out/index_pmc/mode${mode}_info.json" || exit 1
    python tools/pmc_traffic.py gpurun_out --searches 2 --last 2 --nq 1000 --kernel k_ivf_scan \
        --out "gpurun_out/index_pmc/mode$mode.json" > /dev/null || exit 1
    python - "$mode" "$search" <<'PY' || exit 1
import json, os, sys
mode, search = sys.argv[1], sys.argv[2]
p = "gpurun_out/index_pmc/mode%s.json" % mode
d = json.load(open(p)); d["search"] = search; d["mode"] = int(mode)
info = "gpurun_out/index_pmc/mode%s_info.json" % mode
if os.path.exists(info):
    d["nlist"] = json.load(open(info))["nlist"]  # (the last pass's build)
json.dump(d, open(p, "w"), indent=1)
PY
done
rm -rf gpurun_out/pmc1 gpurun_out/pmc2 gpurun_out/pmc3  # raw CSVs: every dispatch of the build too (large)
python - <<'PY'
import glob, json
out = {}
for p in sorted(glob.glob("gpurun_out/index_pmc/mode[0-9].json")):
    d = json.load(open(p)); out[str(d["mode"])] = d
json.dump(out, open("gpurun_out/index_pmc.json", "w"), indent=1)
for m, d in out.items():
    for k, v in d["kernels"].items():
        print(m, d["search"], k, {x: v.get(x) for x in ("launches", "hbm_bytes_per_search", "l2_hit_rate", "mfma_busy_frac")})
PY
