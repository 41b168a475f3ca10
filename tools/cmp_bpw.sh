#!/bin/bash
# C5 (4,096-object sample) and C2 kernel rate at several BMPOW_BLOCKS_PER_WORKER values, same box.
#   usage: tools/cmp_bpw.sh OUTDIR value...
set -e
OUT=${1:?outdir}; shift
mkdir -p "$OUT"
i=0
for v in "$@"; do
  n=bpw${v}_$i; i=$((i + 1))
  BMPOW_BLOCKS_PER_WORKER=$v timeout -k 10 200 python3 bench.py --config c5 --objects 4096 --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/c5_$n.json"
  BMPOW_BLOCKS_PER_WORKER=$v timeout -k 10 200 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/c2_$n.json"
  python3 -c "
import json
a=json.load(open('$OUT/c5_$n.json')); b=json.load(open('$OUT/c2_$n.json'))
print('$n', 'c5', a['value'], a['objects_per_s'], a['roofline']['kernel_ghs'], 'c2', b['value'], b['roofline']['kernel_ghs'], b['wasted_frac'])"
done
