#!/bin/bash
# The whole -m gpu suite and smoke() on the current tree (what the driver runs at round end).
set -euo pipefail
OUT=gpurun_out/r02_suite; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
