#!/bin/bash
set -euo pipefail
OUT=gpurun_out/r02v; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python3 -u tools/shard_latency.py > $OUT/shard_latency.json 2> $OUT/shard_latency.err
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 240 \
  --timeout-method thread > $OUT/pytest_parity.log 2>&1
BMPOW_LIB=variants/nocap/libbmpow_hip.so timeout -k 10 200 python3 -u tools/shard_latency.py > $OUT/shard_latency_nocap.json 2> $OUT/shard_latency_nocap.err
