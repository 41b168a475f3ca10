#!/bin/bash
# Verification kernel A/B on one box: the default build against variants/<name>, resident 500k flood.
#   usage: tools/r02_verify_ab.sh OUTDIR variant...   (variant = default | var_x)
set -euo pipefail
OUT=${1:?outdir}; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
for rep in 1 2; do
for v in "$@"; do
  if [ "$v" = default ]; then L=pybitmessage_amd/lib/libbmpow_hip.so; else L=variants/$v/libbmpow_hip.so; fi
  BMPOW_LIB=$L timeout -k 10 200 python3 bench.py --config verify --steps 10 --warmup 2 --no-cpu-baseline \
    > "$OUT/verify_${v}_$rep.json" 2> "$OUT/verify_${v}_$rep.err"
  python3 -c "import json;d=json.load(open('$OUT/verify_${v}_$rep.json'));r=d['roofline'];print('$v', $rep, d['value'], r['avg_launch_ms'], r['frac'], d['e2e_host_buffers']['objects_per_s'])"
done
done
