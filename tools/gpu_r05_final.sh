# round-5 closing session: GPU tests, 1 % hybrid / nq 1 timelines, the small-batch A/B, then the bench line and its rocprof summary
O=gpurun_out/r05w; mkdir -p $O
bash tools/gpu_r05.sh r05w tests tl_sel1 tl_nq1 && timeout -k 10 500 python -u tools/ab_split.py --dbg --n 50000000 --nqs 1,16 --metrics L2 --modes 1 --splits 2 --sels 1,10 --reps 10 --tunes "X=0" > $O/ps.jsonl 2> $O/ps.err && bash tools/gpu_r05_measure.sh bench
