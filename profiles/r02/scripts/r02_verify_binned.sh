#!/bin/bash
# Binned verification kernel: GPU parity tests (both kernels), then a same-box A/B on resident floods.
set -euo pipefail
OUT=gpurun_out/r02_vbin; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_verify.py -m gpu -x -v --timeout 120 --timeout-method thread \
  > $OUT/pytest_verify.log 2>&1
BMPOW_VBINNED=1 timeout -k 10 300 python3 -u -m pytest tests/test_verify.py -m gpu -x -v --timeout 120 --timeout-method thread \
  > $OUT/pytest_verify_forced_binned.log 2>&1
for rep in 1 2; do
for n in 500000 200000; do
for b in 0 1; do
  BMPOW_VBINNED=$b timeout -k 10 200 python3 bench.py --config verify --objects $n --steps 10 --warmup 2 --no-cpu-baseline \
    > $OUT/verify_n${n}_b${b}_$rep.json 2> $OUT/verify_n${n}_b${b}_$rep.err
  python3 -c "import json;d=json.load(open('$OUT/verify_n${n}_b${b}_$rep.json'));r=d['roofline'];print('n', $n, 'binned', $b, $rep, d['value'], r['avg_launch_ms'], r['frac'])"
done
done
done
