#!/bin/bash
# C5 at full size and default difficulty (100,000 ack/pubkey objects) through worker.PowService.
set -euo pipefail
OUT=gpurun_out/r02_c5svc; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u bench.py --config c5 --service --objects 100000 --steps 1 --warmup 0 --no-cpu-baseline \
  > $OUT/cfg_c5_full_default_service.json 2> $OUT/cfg_c5_full_default_service.err
