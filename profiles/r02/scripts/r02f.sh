#!/bin/bash
# Round-2: verify and address-search legs with their CPU baselines; repeated same-box A/B of the
# per-object-words-in-VGPRs variant.
set -euo pipefail
OUT=${1:?outdir}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --config verify --steps 10 --warmup 2 > "$OUT/verify.json" 2> "$OUT/verify.err"
timeout -k 10 300 python3 bench.py --config addrgen --null-bytes 3 --steps 2 --warmup 1 --cpu-seconds 8 \
  > "$OUT/addrgen_det.json" 2> "$OUT/addrgen_det.err"
timeout -k 10 300 python3 bench.py --config addrgen --addr-mode random --null-bytes 3 --steps 2 --warmup 1 \
  --cpu-seconds 8 > "$OUT/addrgen_random.json" 2> "$OUT/addrgen_random.err"
tools/cmp_variants.sh "$OUT/ab" default variants/var_ihwv default variants/var_ihwv > "$OUT/ab.txt" 2>&1
echo done
