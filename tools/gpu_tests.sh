#!/bin/bash
# The -m gpu suite on the GPU box, one process, each test bounded; plus the gfx950 counter list.
#   usage: tools/gpu_tests.sh OUTDIR [pytest args...]
set -euo pipefail
OUT=${1:?outdir}; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread "$@" \
  > "$OUT/pytest_gpu.log" 2>&1
echo "pytest rc=0" >> "$OUT/pytest_gpu.log"
