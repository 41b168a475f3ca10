#!/bin/bash
# After the per-batch log line: the worker GPU tests and smoke() on the final library build.
set -euo pipefail
OUT=gpurun_out/r02_wcheck; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_worker.py tests/test_gpu_parity.py -m gpu -x -v --timeout 120 \
  --timeout-method thread > $OUT/pytest.log 2>&1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
