set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for d in 256 512 768 1536; do
  timeout -k 10 300 python -u tools/ab_split.py --splits 2 --nqs 1000 --reps 3 --d $d --no-exact --tunes "MQVS_HI_TUNE=2,4,4;MQVS_HI_TUNE=2,4,4,1" >> gpurun_out/dsweep.jsonl 2>> gpurun_out/dsweep.err || exit 1
done
cut -c1-260 gpurun_out/dsweep.jsonl
