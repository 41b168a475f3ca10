#!/bin/bash
# VALU issue counters of bv_pow_kernel on the resident 500k-object flood (one counter group per pass).
set -euo pipefail
OUT=gpurun_out/r02_vpmc${BMPOW_VBINNED:-}; mkdir -p $OUT
export TMPDIR=/tmp
CMD=(python3 bench.py --config verify --steps 4 --warmup 1 --no-cpu-baseline)
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_BUSY_CU_CYCLES SQ_INSTS_VALU \
  SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE --output-format csv -d $OUT/issue -o run -- "${CMD[@]}" \
  > $OUT/issue.json 2> $OUT/issue.err
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VMEM SQ_INSTS_SALU SQ_BUSY_CYCLES --output-format csv -d $OUT/mix -o run -- "${CMD[@]}" \
  > $OUT/mix.json 2> $OUT/mix.err
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- "${CMD[@]}" \
  > $OUT/kt.json 2> $OUT/kt.err
