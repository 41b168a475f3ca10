#!/bin/bash
# PowService A/B: in-tree worker.py (new) against variants/oldsvc (old: a copy of bench.py and the package, here with another SUBMIT_SLICE)
# (variants/oldsvc: a copy of bench.py and the package with the old worker.py), C5 test mode 100k.
set -euo pipefail
OUT=gpurun_out/r02_svc2; mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2 3; do
  for v in new old; do
    B=bench.py; [ $v = old ] && B=variants/oldsvc/bench.py
    timeout -k 10 200 python3 -u $B --config c5 --test-mode --objects 100000 --service --steps 3 --warmup 1 \
      --no-cpu-baseline > $OUT/c5tm_service_${v}_$rep.json 2> $OUT/c5tm_service_${v}_$rep.err
    python3 -c "import json;d=json.load(open('$OUT/c5tm_service_${v}_$rep.json'));print('$v', $rep, d['objects_per_s'], d['roofline']['kernel_busy_frac'])"
  done
done
