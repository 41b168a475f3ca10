#!/bin/bash
# The driver's multi-GPU bench command at 2 and 4 ranks, rehearsed on a one-GPU box: every rank on
# GPU 0 (--share-device), so the values are not scaling numbers -- this checks the launch, the
# claiming over the TCP store, the barriers and the one JSON line on rank 0.
set -euo pipefail
OUT=gpurun_out/r02_scale; mkdir -p $OUT
export TMPDIR=/tmp
for n in 2 4; do
  timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29500 + n)) bench.py --gpus $n --steps 2 --warmup 1 --share-device \
    > $OUT/bench_n$n.json 2> $OUT/bench_n$n.err
done
