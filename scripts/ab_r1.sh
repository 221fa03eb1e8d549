# A/B on one box: the round-1 tree (ab_r1/, built in-tree) against this tree, N=1 bench
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  (cd ab_r1 && timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-smoke) > gpurun_out/ab_r1_$i.log 2>&1 || exit 1
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --batches 4 --no-uncoalesced --no-smoke > gpurun_out/ab_r2_$i.log 2>&1 || exit 1
done
for f in gpurun_out/ab_r1_*.log gpurun_out/ab_r2_*.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f)"; done
