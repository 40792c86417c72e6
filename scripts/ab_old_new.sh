# Same-box A/B of the headline: this tree against an older build checked out
# (git worktree) and built under _ab_old/, alternating, 3 pairs.
set -e
B="--steps 40 --warmup 10 --no-cpu --no-aux --no-sub --no-c4-check"
for i in 1 2 3; do
  (cd _ab_old && timeout -k 10 200 python bench.py $B > ../gpurun_out/ab_old_$i.log 2>&1)
  timeout -k 10 200 python bench.py $B > gpurun_out/ab_new_$i.log 2>&1
done
