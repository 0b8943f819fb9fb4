# short tiles for gathered main segments: tests, then A/B (MQVS_HI_SMALL_MAIN=0 = 256-row tiles)
O=gpurun_out/r05u; mkdir -p $O
bash tools/gpu_r05.sh r05u tests tl_sel1 && timeout -k 10 500 python -u tools/ab_split.py --dbg --n 50000000 --nqs 1,16 --metrics L2,Cosine --modes 1 --splits 2 --sels 1,10,50 --reps 10 --tunes "X=0;MQVS_HI_SMALL_MAIN=0;X=0;MQVS_HI_SMALL_MAIN=0" > $O/sm.jsonl 2> $O/sm.err
