#!/bin/bash
# Verification kernel, resident 500k flood: group layout period A/B (BMPOW_VSNAKE, 0 = sorted order).
set -euo pipefail
OUT=${1:?outdir}; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
for rep in 1 2; do
for p in "$@"; do
  BMPOW_VSNAKE=$p timeout -k 10 200 python3 bench.py --config verify --steps 10 --warmup 2 --no-cpu-baseline \
    > "$OUT/verify_s${p}_$rep.json" 2> "$OUT/verify_s${p}_$rep.err"
  python3 -c "import json;d=json.load(open('$OUT/verify_s${p}_$rep.json'));r=d['roofline'];print('snake', $p, $rep, d['value'], r['avg_launch_ms'], r['frac'])"
done
done
