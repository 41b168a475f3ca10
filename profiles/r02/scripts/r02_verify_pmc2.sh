#!/bin/bash
# bv_pow_kernel memory-side and instruction-fetch counters (one group per pass), plus the counter list.
set -uo pipefail
OUT=gpurun_out/r02_vpmc2; mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1
CMD=(python3 bench.py --config verify --steps 3 --warmup 1 --no-cpu-baseline)
timeout -s KILL 120 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum --output-format csv -d $OUT/tcp -o run -- "${CMD[@]}" \
  > $OUT/tcp.json 2> $OUT/tcp.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/tcc -o run -- "${CMD[@]}" \
  > $OUT/tcc.json 2> $OUT/tcc.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_IFETCH SQ_INSTS_VMEM SQ_WAIT_ANY SQ_WAVES SQ_INST_LEVEL_VMEM SQ_ACCUM_PREV_HIRES --output-format csv -d $OUT/sq -o run -- "${CMD[@]}" \
  > $OUT/sq.json 2> $OUT/sq.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS --output-format csv -d $OUT/ic -o run -- "${CMD[@]}" \
  > $OUT/ic.json 2> $OUT/ic.err || exit 1
