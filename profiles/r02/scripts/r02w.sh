#!/bin/bash
set -euo pipefail
OUT=gpurun_out/r02w; mkdir -p $OUT
export TMPDIR=/tmp
BMPOW_LIB=variants/nocap/libbmpow_hip.so timeout -k 10 200 python3 -u tools/shard_latency.py > $OUT/shard_latency_nocap.json 2> $OUT/shard_latency_nocap.err
