#!/bin/bash
set -euo pipefail
OUT=gpurun_out/r02z; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_worker.py -m gpu -x -v --timeout 120 --timeout-method thread \
  > $OUT/pytest_worker.log 2>&1
