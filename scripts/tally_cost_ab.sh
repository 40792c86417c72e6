# The headline with and without the tally in the step (bench.py --no-tally),
# alternating on one box, 2 pairs: what the tally beside the verifications costs.
set -e
B="--steps 400 --warmup 10 --no-cpu --no-aux --no-sub --no-c4-check"
for i in 1 2; do
  timeout -k 10 200 python bench.py $B > gpurun_out/tc_tally_$i.log 2>&1
  timeout -k 10 200 python bench.py $B --no-tally > gpurun_out/tc_notally_$i.log 2>&1
done
