#!/bin/bash
# BASELINE C5 at full size and protocol-default difficulty: 100,000 ack/pubkey objects, one pass.
set -euo pipefail
OUT=gpurun_out/r02y; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u bench.py --config c5 --objects 100000 --steps 1 --warmup 0 --no-cpu-baseline \
  > $OUT/c5_full.json 2> $OUT/c5_full.err
