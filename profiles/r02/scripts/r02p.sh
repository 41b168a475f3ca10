#!/bin/bash
set -euo pipefail
OUT=${1:?outdir}
mkdir -p "$OUT"
export TMPDIR=/tmp
for rep in 1 2; do
for a in 32768 1000000; do
  timeout -k 10 300 python3 bench.py --config c5 --test-mode --objects 100000 --service --service-add-per-step $a \
    --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/svc_${a}_$rep.json" 2> "$OUT/svc_${a}_$rep.err"
done
done
echo done
