#!/bin/bash
# Verification kernel A/B: GPU parity of the in-tree build (both kernels), then resident floods for the
# in-tree build and variants/<name> with the binned kernel off/on (BMPOW_VBINNED).
#   usage: tools/r02_verify_ab2.sh OUTDIR variant...
set -euo pipefail
OUT=${1:?outdir}; shift
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_verify.py -m gpu -x -v --timeout 120 --timeout-method thread \
  > $OUT/pytest_verify.log 2>&1
BMPOW_VBINNED=1 timeout -k 10 300 python3 -u -m pytest tests/test_verify.py -m gpu -x -v --timeout 120 --timeout-method thread \
  > $OUT/pytest_verify_binned.log 2>&1
BMPOW_VBINNED=0 timeout -k 10 300 python3 -u -m pytest tests/test_verify.py -m gpu -x -v --timeout 120 --timeout-method thread \
  > $OUT/pytest_verify_unbinned.log 2>&1
for rep in 1 2; do
for v in default "$@"; do
  if [ "$v" = default ]; then L=pybitmessage_amd/lib/libbmpow_hip.so; else L=variants/$v/libbmpow_hip.so; fi
  for n in 500000 200000; do
  for b in 0 1; do
    BMPOW_LIB=$L BMPOW_VBINNED=$b timeout -k 10 200 python3 bench.py --config verify --objects $n --steps 10 --warmup 2 \
      --no-cpu-baseline > $OUT/verify_${v}_n${n}_b${b}_$rep.json 2> $OUT/verify_${v}_n${n}_b${b}_$rep.err
    python3 -c "import json;d=json.load(open('$OUT/verify_${v}_n${n}_b${b}_$rep.json'));r=d['roofline'];print('$v', $n, 'binned', $b, $rep, d['value'], r['avg_launch_ms'], r['frac'])"
  done
  done
done
done
