#!/bin/bash
# Round 2: native service -- new GPU tests, then C5 test-mode 100k objects: service vs run_batch.
set -euo pipefail
OUT=gpurun_out/r02q; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_worker.py -m gpu -x -v --timeout 120 \
  --timeout-method thread -k "service or powservice" > $OUT/pytest_service.log 2>&1
timeout -k 10 200 python3 -u bench.py --config c5 --test-mode --objects 100000 --service --steps 3 --warmup 1 \
  > $OUT/c5_service.json 2> $OUT/c5_service.err
timeout -k 10 200 python3 -u bench.py --config c5 --test-mode --objects 100000 --run-batch --steps 3 --warmup 1 \
  > $OUT/c5_runbatch.json 2> $OUT/c5_runbatch.err
timeout -k 10 200 python3 -u bench.py --config c5 --service --steps 1 --warmup 1 \
  > $OUT/c5_default_service.json 2> $OUT/c5_default_service.err
