#!/bin/bash
# round-5 first GPU pass: the whole -m gpu suite, a short bench line, the
# configs[4] gather-source A/B.  Outputs gpurun_out/r5a/.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5a
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -q --maxfail=5 --timeout 300 --timeout-method thread > $O/tests.log 2>&1
echo "tests_rc=$?"; tail -3 $O/tests.log
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-index --no-configs --no-config1-points --no-cpu > $O/bench.json 2> $O/bench.err
echo "bench_rc=$?"
timeout -k 10 400 python tools/gather_source_ab.py > $O/gather_ab.jsonl 2> $O/gather_ab.err
echo "gather_rc=$?"
timeout -k 10 500 python -u tools/ab_split.py --dbg --nqs 1000 --metrics Cosine --modes 1 --splits 2 --reps 5 --no-exact \
  --tunes 'MQVS_P4M_DIAG=0;MQVS_P4M_DIAG=1;MQVS_P4M_DIAG=4;MQVS_P4M_DIAG=6;MQVS_P4M_DIAG=7;MQVS_P4M_DIAG=0' > $O/p4m_diag.jsonl 2> $O/p4m_diag.err
echo "diag_rc=$?"
exit 0
