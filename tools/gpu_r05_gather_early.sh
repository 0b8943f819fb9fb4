# gather list compacted before the count reaches the host: tests, timeline, A/B (MQVS_GATHER_EARLY=0 = after)
O=gpurun_out/r05x; mkdir -p $O
bash tools/gpu_r05.sh r05x tests tl_sel1 && timeout -k 10 600 python -u tools/ab_split.py --dbg --n 50000000 --nqs 1,16 --metrics L2,Cosine --modes 1 --splits 2 --sels 1,10,80 --reps 10 --tunes "X=0;MQVS_GATHER_EARLY=0;X=0;MQVS_GATHER_EARLY=0" > $O/ge.jsonl 2> $O/ge.err
