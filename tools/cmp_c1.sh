#!/bin/bash
# C1 (one object via proofofwork.run) and C3 kernel rate of alternative builds (BMPOW_LIB), same box.
#   usage: tools/cmp_c1.sh OUTDIR variant...   (variant = default | variants/<name>)
set -e
OUT=${1:?outdir}; shift
mkdir -p "$OUT"
i=0
for v in "$@"; do
  if [ "$v" = default ]; then L=pybitmessage_amd/lib/libbmpow_hip.so; else L=$v/libbmpow_hip.so; fi
  n=$(basename "$v")_$i; i=$((i + 1))
  BMPOW_LIB=$L timeout -k 10 120 python3 bench.py --config c1 --steps 40 --warmup 3 --no-cpu-baseline > "$OUT/c1_$n.json"
  BMPOW_LIB=$L timeout -k 10 120 python3 bench.py --config c3 --c3-log2 35 --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/c3_$n.json"
  python3 -c "
import json
a=json.load(open('$OUT/c1_$n.json')); b=json.load(open('$OUT/c3_$n.json'))
print('$n', 'c1', a['value'], a['wasted_frac'], a['ms_per_step'], 'c3', b['roofline']['kernel_ghs'])"
done
