#!/bin/bash
# Re-entry check of the restored tree: the -m gpu suite, then the default bench line.
set -euo pipefail
OUT=gpurun_out/r02_reentry; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1
timeout -k 10 400 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err
