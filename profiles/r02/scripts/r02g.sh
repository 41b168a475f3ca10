#!/bin/bash
set -euo pipefail
OUT=${1:?outdir}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_verify.py -m gpu -x -v --timeout 240 --timeout-method thread \
  > "$OUT/pytest_verify.log" 2>&1
timeout -k 10 300 python3 bench.py --config verify --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/verify.json" 2> "$OUT/verify.err"
echo done
