#!/bin/bash
set -euo pipefail
OUT=${1:?outdir}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_verify.py -m gpu -x -v --timeout 240 --timeout-method thread \
  > "$OUT/pytest_verify.log" 2>&1
timeout -k 10 300 python3 bench.py --config verify --steps 10 --warmup 2 > "$OUT/verify.json" 2> "$OUT/verify.err"
tools/cmp_variants.sh "$OUT/ab" default variants/var_w5 variants/var_w6 default > "$OUT/ab.txt" 2>&1
echo done
