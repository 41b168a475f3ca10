#!/bin/bash
# Final-tree check: the -m gpu suite, smoke(), the default bench line, and the rocprofv3 kernel
# statistics of the same default command.
set -euo pipefail
OUT=gpurun_out/r02_final; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
timeout -k 10 400 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 bench.py \
  > $OUT/bench_under_rocprof.json 2> $OUT/bench_under_rocprof.err
