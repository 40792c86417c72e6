#!/bin/bash
# N > 1 bench path rehearsed on one GPU: 2 and 3 ranks sharing the card,
# gloo (host) collectives; checks the sharded verify + partitioned tally run
set -o pipefail
mkdir -p gpurun_out
for n in 2 3; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --steps 5 --warmup 1 --dist-backend gloo --batch 262144 > gpurun_out/rehearse_$n.json 2> gpurun_out/rehearse_$n.err || { tail -30 gpurun_out/rehearse_$n.err; exit 1; }
  cut -c1-600 gpurun_out/rehearse_$n.json
done
