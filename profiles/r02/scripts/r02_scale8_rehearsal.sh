#!/bin/bash
# The driver's N=8 bench command rehearsed on a one-GPU box: 8 ranks all on GPU 0 (--share-device),
# so the value is not a scaling number; checks launch, claiming, barriers and rank 0's one JSON line.
set -euo pipefail
OUT=gpurun_out/r02_scale8; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port 29581 bench.py --gpus 8 --steps 1 --warmup 1 --share-device > $OUT/bench_n8.json 2> $OUT/bench_n8.err
