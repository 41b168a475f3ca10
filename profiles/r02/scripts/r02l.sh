#!/bin/bash
set -euo pipefail
OUT=${1:?outdir}
mkdir -p "$OUT"
export TMPDIR=/tmp
tools/cmp_variants.sh "$OUT/ab" default variants/var_w5i64 variants/var_w5sst variants/var_w5st default > "$OUT/ab.txt" 2>&1
timeout -k 10 300 python3 bench.py --config c5 --test-mode --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/c5tm_batch.json" 2> "$OUT/c5tm_batch.err"
timeout -k 10 300 python3 bench.py --config c5 --test-mode --objects 100000 --service --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/c5tm_service.json" 2> "$OUT/c5tm_service.err"
echo done
