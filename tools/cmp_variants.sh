#!/bin/bash
# C3 kernel rate of alternative builds of libbmpow_hip.so (BMPOW_LIB) on the same box.
#   usage: tools/cmp_variants.sh OUTDIR variant...   (variant = default | build/<name>)
set -e
OUT=${1:?outdir}; shift
mkdir -p "$OUT"
for v in "$@"; do
  if [ "$v" = default ]; then L=pybitmessage_amd/lib/libbmpow_hip.so; else L=$v/libbmpow_hip.so; fi
  n=$(basename "$v")
  BMPOW_LIB=$L timeout -k 10 120 python3 bench.py --config c3 --c3-log2 35 --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/c3_$n.json"
  python3 -c "import json;d=json.load(open('$OUT/c3_$n.json'));r=d['roofline'];print('$n', r['kernel_ghs'], r['avg_launch_ms'])"
done
