#!/bin/bash
# PMC passes for ar_search_kernel (address search, 3 null bytes), one counter group per
# rocprofv3 run, no tracing domains beside --pmc.   usage: tools/profile_pmc_addr.sh OUTDIR
set -euo pipefail
OUT=${1:?outdir}
mkdir -p "$OUT"
export TMPDIR=/tmp
CMD=(python3 bench.py --config addrgen --null-bytes 3 --steps 1 --warmup 0 --no-cpu-baseline)
pass() {
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- "${CMD[@]}" \
    > "$OUT/$name.bench.json" 2> "$OUT/$name.err"
}
pass instr SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_LDS GRBM_GUI_ACTIVE
pass busy SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE
echo "pmc passes done: $OUT"
