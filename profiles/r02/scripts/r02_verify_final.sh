#!/bin/bash
# Verification leg after the binned kernel: GPU parity tests, the bench line (with its CPU baseline),
# and the rocprofv3 kernel statistics of the same command.
set -euo pipefail
OUT=gpurun_out/r02_vfinal; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_verify.py -m gpu -x -v --timeout 120 --timeout-method thread \
  > $OUT/pytest_verify.log 2>&1
timeout -k 10 300 python3 bench.py --config verify > $OUT/cfg_verify.json 2> $OUT/cfg_verify.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- \
  python3 bench.py --config verify --no-cpu-baseline > $OUT/kt_bench.json 2> $OUT/kt.err
