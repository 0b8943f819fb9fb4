#!/bin/bash
# round-5 pass c: tests touched since pass b, kernel timelines of the 1 %
# gathered search (50M x 768 L2, nq 1) and of nq 1 over 10M x 768 cosine,
# the gather A/B again.  Outputs gpurun_out/r5c/.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5c
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_concurrency.py tests/test_gpu_batch.py tests/test_gpu_parity.py -m gpu -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
echo "tests_rc=$?"; tail -3 $O/tests.log
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/tr_sel1" -o run --output-format csv \
    -- python3 "$GRAFT_REPO_ROOT/tools/pmc_search.py" --nq 1 --n 50000000 --metric L2 --selectivity 1 --searches 4 \
    > "$GRAFT_REPO_ROOT/$O/tr_sel1.log" 2>&1 ) || { echo "trace sel1 failed"; exit 1; }
python3 tools/timeline.py $O/tr_sel1/run_kernel_trace.csv --start k_chunk_count --nth -1
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/tr_nq1" -o run --output-format csv \
    -- python3 "$GRAFT_REPO_ROOT/tools/pmc_search.py" --nq 1 --searches 4 \
    > "$GRAFT_REPO_ROOT/$O/tr_nq1.log" 2>&1 ) || { echo "trace nq1 failed"; exit 1; }
python3 tools/timeline.py $O/tr_nq1/run_kernel_trace.csv --start k_query_prep --nth -1
timeout -k 10 400 python tools/gather_source_ab.py --nq 1,16 --sel 1,10 > $O/gather_ab.jsonl 2> $O/gather_ab.err
echo "gather_rc=$?"
exit 0
