#!/bin/bash
set -euo pipefail
OUT=${1:?outdir}
mkdir -p "$OUT"
export TMPDIR=/tmp
tools/cmp_variants.sh "$OUT/ab" default variants/var_w5 variants/var_w5ilp variants/var_w5i16 variants/var_w5bias variants/var_w5 default > "$OUT/ab.txt" 2>&1
echo done
