#!/bin/bash
# C2 and the C5 sample at several per-launch trial budgets (bench.py --step-trials), same box.
#   usage: tools/cmp_step.sh OUTDIR log2...
set -e
OUT=${1:?outdir}; shift
mkdir -p "$OUT"
i=0
for l in "$@"; do
  n=s${l}_$i; i=$((i + 1))
  timeout -k 10 200 python3 bench.py --config c5 --objects 4096 --steps 1 --warmup 0 --no-cpu-baseline --step-trials $((1 << l)) > "$OUT/c5_$n.json"
  timeout -k 10 200 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --step-trials $((1 << l)) > "$OUT/c2_$n.json"
  python3 -c "
import json
a=json.load(open('$OUT/c5_$n.json')); b=json.load(open('$OUT/c2_$n.json'))
print('$n', 'c5', a['value'], a['objects_per_s'], a['roofline']['kernel_ghs'], a['roofline']['kernel_busy_frac'], 'c2', b['value'], b['roofline']['kernel_ghs'], b['roofline']['kernel_busy_frac'])"
done
