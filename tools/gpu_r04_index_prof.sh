#!/bin/bash
# kernel-trace breakdown of index searches (configs[2], mode 3 nprobe 1 and
# mode 2 nprobe 8): rocprofv3 --kernel-trace --stats over tools/index_sweep.py.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04_index_prof
mkdir -p $O
for spec in "3:nprobe=1" "2:nprobe=8"; do
  mode=${spec%%:*}; search=${spec#*:}
  ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/m$mode" -o run --output-format csv \
      -- python3 "$GRAFT_REPO_ROOT/tools/index_sweep.py" --mode "$mode" --search "$search" --reps 5 \
      > "$GRAFT_REPO_ROOT/$O/m$mode.jsonl" 2> "$GRAFT_REPO_ROOT/$O/m$mode.err" ) || { echo "prof m$mode failed"; tail -5 $O/m$mode.err; exit 1; }
  python3 - "$O/m$mode/run_kernel_trace.csv" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
# the last 5 searches: kernels after the last "k_plan" group... simple: aggregate kernels by name over the whole run,
# and also the per-kernel time of the final search window (after the last k_to_bf16 launch)
idx = [i for i, r in enumerate(rows) if "k_to_bf16" in r["Kernel_Name"]]
last = rows[idx[-1]:] if idx else rows
agg = collections.OrderedDict()
for r in last:
    n = r["Kernel_Name"].split("(")[0][:90]
    agg.setdefault(n, 0.0)
    agg[n] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
t0 = int(last[0]["Start_Timestamp"]); t1 = int(last[-1]["End_Timestamp"])
print("last search: span %.3f ms, kernels %.3f ms" % ((t1 - t0) / 1e6, sum(agg.values())))
for n, v in agg.items(): print("  %.4f  %s" % (v, n))
PY
done
exit 0
