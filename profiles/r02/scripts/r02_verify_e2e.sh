#!/bin/bash
# Verification end to end from host buffers (and resident), the GPU verify tests first.
set -euo pipefail
OUT=gpurun_out/r02_ve2e; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_verify.py -m gpu -x -v --timeout 120 --timeout-method thread \
  > $OUT/pytest_verify.log 2>&1
for rep in 1 2; do
  timeout -k 10 300 python3 bench.py --config verify --no-cpu-baseline > $OUT/cfg_verify_$rep.json 2> $OUT/cfg_verify_$rep.err
  python3 -c "import json;d=json.load(open('$OUT/cfg_verify_$rep.json'));e=d['e2e_host_buffers'];print($rep, d['value'], e['objects_per_s'], e['seconds'], e['parts'])"
done
