set -e
B="--no-cpu --no-aux --no-sub --no-c4-check"
for i in 1 2; do
  for k in 20 100 400; do
    timeout -k 10 200 python bench.py --steps $k --warmup 5 $B > gpurun_out/steps_${k}_$i.log 2>&1
  done
done
