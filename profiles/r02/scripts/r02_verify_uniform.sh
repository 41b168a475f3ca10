#!/bin/bash
set -euo pipefail
OUT=gpurun_out/r02_vuni; mkdir -p $OUT
export TMPDIR=/tmp
BMPOW_VBINNED=0 timeout -k 10 300 python3 tools/verify_uniform.py > $OUT/unbinned.jsonl 2> $OUT/unbinned.err
BMPOW_VBINNED=1 timeout -k 10 300 python3 tools/verify_uniform.py > $OUT/binned.jsonl 2> $OUT/binned.err
