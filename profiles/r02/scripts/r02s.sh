#!/bin/bash
set -euo pipefail
OUT=gpurun_out/r02s; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/service_timeline.py > $OUT/timeline.json 2> $OUT/timeline.err
