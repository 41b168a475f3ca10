#!/bin/bash
# Counters of the verification kernel (resident 500k flood) and of the address-search kernel (both
# modes, one search each): VALU issue, then FETCH_SIZE and WRITE_SIZE in passes of their own.
set -euo pipefail
OUT=gpurun_out/r02_pmc2; mkdir -p $OUT
export TMPDIR=/tmp
ISSUE="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_BUSY_CU_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE"
run() {  # name, then the command
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc $ISSUE --output-format csv -d $OUT/$name/issue -o run -- "$@" > $OUT/$name.issue.json 2> $OUT/$name.issue.err
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/$name/fetch -o run -- "$@" > $OUT/$name.fetch.json 2> $OUT/$name.fetch.err
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/$name/write -o run -- "$@" > $OUT/$name.write.json 2> $OUT/$name.write.err
}
run verify python3 bench.py --config verify --steps 3 --warmup 1 --no-cpu-baseline
run addr_det python3 bench.py --config addrgen --steps 1 --warmup 0 --no-cpu-baseline
run addr_random python3 bench.py --config addrgen --addr-mode random --steps 1 --warmup 0 --no-cpu-baseline
