#!/bin/bash
# PowService with array-backed results: the worker GPU tests, then C5 at test-mode difficulty (100k
# objects) through PowService, run_batch and the raw batch, twice each, same box.
set -euo pipefail
OUT=gpurun_out/r02_svc; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_worker.py -m gpu -x -v --timeout 120 --timeout-method thread \
  > $OUT/pytest_worker.log 2>&1
for rep in 1 2; do
  for leg in service run-batch batch; do
    flag=""; [ $leg = service ] && flag=--service; [ $leg = run-batch ] && flag=--run-batch
    timeout -k 10 200 python3 -u bench.py --config c5 --test-mode --objects 100000 $flag --steps 3 --warmup 1 \
      --no-cpu-baseline > $OUT/c5tm_${leg}_$rep.json 2> $OUT/c5tm_${leg}_$rep.err
    python3 -c "import json;d=json.load(open('$OUT/c5tm_${leg}_$rep.json'));print('$leg', $rep, d['objects_per_s'], d['value'], d['roofline']['kernel_busy_frac'])"
  done
done
