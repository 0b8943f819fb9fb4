#!/bin/bash
# round-5 GPU steps: tools/gpu_r05.sh OUTDIR step... (tests | tests_quick |
# tl_sel1 | tl_nq1 | bench_quick | bench | gather_ab).  Each step has its own
# time limit; the first failing step ends the call.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/$1; shift
IDX_TUNES=${IDX_TUNES:-";MQVS_IVF_CHUNK=256;MQVS_IVF_CHUNK=128;MQVS_IVF_CHUNK=256,MQVS_IVF_GRID=2048;MQVS_IVF_CHUNK=128,MQVS_IVF_GRID=4096"}
mkdir -p $O
trace() {  # name, args...
  local name=$1; shift
  ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/$name" -o run --output-format csv \
      -- python3 "$GRAFT_REPO_ROOT/tools/pmc_search.py" "$@" > "$GRAFT_REPO_ROOT/$O/$name.log" 2>&1 )
}
for step in "$@"; do
  case $step in
    tests) timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
           rc=$?; tail -4 $O/tests.log; [ $rc -eq 0 ] || exit $rc ;;
    tl_sel1) trace tr_sel1 --nq 1 --n 50000000 --metric L2 --selectivity 1 --searches 4 || exit 1
             python3 tools/timeline.py $O/tr_sel1/run_kernel_trace.csv --start k_chunk_count --nth -1 ;;
    tl_nq1) trace tr_nq1 --nq 1 --searches 4 || exit 1
            python3 tools/timeline.py $O/tr_nq1/run_kernel_trace.csv --start k_query_prep --nth -1 ;;
    tl_idx3|tl_idx2)  # one index search (mode 3 nprobe 1 / mode 2 nprobe 1), last of 3
            m=${step#tl_idx}
            ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/tr_idx$m" -o run --output-format csv \
                -- python3 "$GRAFT_REPO_ROOT/tools/index_search_run.py" --mode $m --search nprobe=1 --searches 3 \
                > "$GRAFT_REPO_ROOT/$O/tr_idx$m.log" 2>&1 ) || exit 1
            python3 tools/timeline.py $O/tr_idx$m/run_kernel_trace.csv --start k_to_bf16 --nth -1 ;;
    idx_ab) for m in 3 2; do
              timeout -k 10 400 python -u tools/index_scan_ab.py --mode $m --search "${IDX_SEARCH:-nprobe=1}" --tunes "$IDX_TUNES" > $O/idx_ab$m.jsonl 2> $O/idx_ab$m.err || exit 1
              cat $O/idx_ab$m.jsonl
            done ;;
    bench_quick) timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-index --no-configs --no-config1-points --no-cpu > $O/bench_quick.json 2> $O/bench_quick.err || exit 1
                 python3 -c "import json;d=json.loads(open('$O/bench_quick.json').readlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline']);print([ (x['nq'],x['ms_per_search'],x['hbm_frac_end_to_end']) for x in d['small_batch']])" ;;
    bench) timeout -k 10 900 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 1 ;;
    gather_ab) timeout -k 10 400 python tools/gather_source_ab.py --nq 1,16 --sel 1,10 > $O/gather_ab.jsonl 2> $O/gather_ab.err || exit 1 ;;
    seg_ab) timeout -k 10 600 python -u tools/ab_split.py --dbg --nqs 1 --metrics Cosine --modes 1 --splits 2 --reps 10 \
              --tunes 'MQVS_SEG=8,4,65536;MQVS_SEG=8,16,65536;MQVS_SEG=8,64,65536;MQVS_SEG=32,64,65536;MQVS_SEG=8,4,65536' \
              > $O/seg_ab_nq1.jsonl 2> $O/seg_ab_nq1.err || exit 1
            timeout -k 10 600 python -u tools/ab_split.py --dbg --nqs 16 --metrics Cosine --modes 1 --splits 2 --reps 10 \
              --tunes 'MQVS_SEG=4,4,16384;MQVS_SEG=4,16,16384;MQVS_SEG=8,64,16384;MQVS_SEG=8,64,65536;MQVS_SEG=4,4,16384' \
              > $O/seg_ab_nq16.jsonl 2> $O/seg_ab_nq16.err || exit 1
            python3 -c "
import json
for f in ('$O/seg_ab_nq1.jsonl','$O/seg_ab_nq16.jsonl'):
    for l in open(f):
        d=json.loads(l); print(d['tune'], d['nq'], 'wall', d['wall_ms'], 'med', d.get('wall_med_ms'), 'main', d['main_ms'], 'segs', d['segments'], 'eq', d['bitwise_eq_exact'])
" ;;
    qprep_ab) timeout -k 10 120 ./tools/bin/qprep_sum_ab > $O/qprep_sum_ab.jsonl 2> $O/qprep_sum_ab.err || exit 1
              cat $O/qprep_sum_ab.jsonl ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
  echo "step $step ok"
done
exit 0
