#!/bin/bash
set -euo pipefail
OUT=${1:?outdir}
mkdir -p "$OUT"
export TMPDIR=/tmp
tools/gpu_tests.sh "$OUT"
for p in "" "--run-batch" "--service"; do
  n=c5tm${p//-/_}
  timeout -k 10 300 python3 bench.py --config c5 --test-mode --objects 100000 $p --steps 1 --warmup 1 --no-cpu-baseline \
    > "$OUT/$n.json" 2> "$OUT/$n.err"
done
timeout -k 10 300 python3 bench.py --config c2 --run-batch --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/c2_run_batch.json" 2> "$OUT/c2_run_batch.err"
echo done
