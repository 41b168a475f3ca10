#!/bin/bash
set -euo pipefail
OUT=gpurun_out/r02x; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python3 -u tools/shard_latency.py > $OUT/shard_latency.json 2> $OUT/shard_latency.err
BMPOW_LIB=variants/nocap/libbmpow_hip.so timeout -k 10 200 python3 -u tools/shard_latency.py > $OUT/shard_latency_nocap.json 2> $OUT/shard_latency_nocap.err
