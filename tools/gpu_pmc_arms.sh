#!/bin/bash
# PMC passes (tools/gpu_pmc.sh) over ab_split.py, one set per arm:
#   bash tools/gpu_pmc_arms.sh "<ab args>" "TAG1:ENV=V ENV2=V" "TAG2:..." ...
# Each arm's passes land in gpurun_out/pmc_<TAG>/pmc{1,2,3}.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
ARGS="$1"; shift
for arm in "$@"; do
  tag="${arm%%:*}"; envs="${arm#*:}"
  env $envs bash tools/gpu_pmc.sh python tools/ab_split.py $ARGS || exit 1
  mkdir -p "gpurun_out/pmc_$tag" && mv gpurun_out/pmc1 gpurun_out/pmc2 gpurun_out/pmc3 gpurun_out/pmc*.log "gpurun_out/pmc_$tag/" || exit 1
done
