#!/bin/bash
# round-5 second pass: the failing tests again, the p4m DMA-placement A/B, the
# configs[4] gather-source A/B.  Outputs gpurun_out/r5b/.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5b
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_concurrency.py tests/test_gpu_bench_loopback.py -m gpu -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
echo "tests_rc=$?"; tail -3 $O/tests.log
timeout -k 10 600 python -u tools/ab_split.py --dbg --nqs 1000 --metrics Cosine,L2 --modes 1 --splits 2 --reps 5 \
  --tunes 'MQVS_P4M_PL=0;MQVS_P4M_PL=1;MQVS_P4M_PL=2;MQVS_P4M_PL=3;MQVS_P4M_PL=0' > $O/p4m_pl.jsonl 2> $O/p4m_pl.err
echo "pl_rc=$?"
timeout -k 10 400 python tools/gather_source_ab.py > $O/gather_ab.jsonl 2> $O/gather_ab.err
echo "gather_rc=$?"
exit 0
