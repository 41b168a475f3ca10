#!/bin/bash
# Round 2: PowService with submit records and sliced submission -- C5 test mode, 100k objects.
set -euo pipefail
OUT=gpurun_out/r02r; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python3 -u bench.py --config c5 --test-mode --objects 100000 --service --steps 3 --warmup 1 \
  --no-cpu-baseline > $OUT/c5_service.json 2> $OUT/c5_service.err
timeout -k 10 200 python3 -u -m pytest tests/test_worker.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 \
  --timeout-method thread -k "service" > $OUT/pytest_service.log 2>&1
timeout -k 10 200 python3 -u bench.py --config c5 --test-mode --objects 100000 --run-batch --steps 3 --warmup 1 \
  --no-cpu-baseline > $OUT/c5_runbatch.json 2> $OUT/c5_runbatch.err
