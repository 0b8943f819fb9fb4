# probe select with LDS-staged keys: tests, then A/B (MQVS_PS_STAGE=0 = keys re-read from L2 per pass)
O=gpurun_out/r05v; mkdir -p $O
bash tools/gpu_r05.sh r05v tests tl_sel1 && timeout -k 10 500 python -u tools/ab_split.py --dbg --n 50000000 --nqs 1,16 --metrics L2,Cosine --modes 1 --splits 2 --sels 1,10 --reps 10 --tunes "X=0;MQVS_PS_STAGE=0;X=0;MQVS_PS_STAGE=0" > $O/ps.jsonl 2> $O/ps.err
