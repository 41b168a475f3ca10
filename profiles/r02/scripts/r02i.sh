#!/bin/bash
set -euo pipefail
OUT=${1:?outdir}
mkdir -p "$OUT"
export TMPDIR=/tmp
tools/cmp_variants.sh "$OUT/ab" default variants/var_w5 variants/var_w5s variants/var_w6s default variants/var_w5 variants/var_w5s > "$OUT/ab.txt" 2>&1
echo done
