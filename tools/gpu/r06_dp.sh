#!/bin/bash
# round 6: the N > 1 bench path rehearsed on the one-GPU box (gloo ranks sharing the card), final tree
set -o pipefail
O=gpurun_out/r06dp
mkdir -p $O
PFM_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 > $O/n2.json 2> $O/n2.err || { tail -30 $O/n2.err; exit 1; }
tail -1 $O/n2.json | cut -c1-600
