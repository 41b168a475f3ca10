#!/bin/bash
# Round-2 bench lines for the BASELINE configs not re-measured since the 5-wave kernel: C3 (2^38
# nonces, one GPU), C4 (64 objects at 20x difficulty), C1 (one object via bmpow_search), plus the
# rocprofv3 kernel statistics of the C3 command.
set -euo pipefail
OUT=gpurun_out/r02_cfg; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --config c3 --c3-log2 38 --steps 1 --warmup 0 --no-cpu-baseline > $OUT/cfg_c3.json 2> $OUT/cfg_c3.err
timeout -k 10 300 python3 bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/cfg_c4.json 2> $OUT/cfg_c4.err
timeout -k 10 300 python3 bench.py --config c1 --no-cpu-baseline > $OUT/cfg_c1.json 2> $OUT/cfg_c1.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_c3 -o run -- \
  python3 bench.py --config c3 --c3-log2 36 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/kt_c3.json 2> $OUT/kt_c3.err
