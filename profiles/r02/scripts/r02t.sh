#!/bin/bash
set -euo pipefail
OUT=gpurun_out/r02t; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/service_timeline.py > $OUT/timeline.json 2> $OUT/timeline.err
timeout -k 10 200 python3 -u bench.py --config c5 --test-mode --objects 100000 --service --steps 3 --warmup 1 \
  --no-cpu-baseline > $OUT/c5_service.json 2> $OUT/c5_service.err
timeout -k 10 200 python3 -u -m pytest tests/test_worker.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 \
  --timeout-method thread -k "service" > $OUT/pytest_service.log 2>&1
