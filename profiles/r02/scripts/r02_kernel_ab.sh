#!/bin/bash
# Round-2 search-kernel A/B + VALU issue counters + default bench line.
#   usage: tools/r02_kernel_ab.sh OUTDIR
set -euo pipefail
OUT=${1:?outdir}
mkdir -p "$OUT"
export TMPDIR=/tmp
tools/cmp_variants.sh "$OUT/ab" default variants/var_add64 variants/var_ihwv > "$OUT/ab.txt" 2>&1
CMD=(python3 bench.py --config c3 --c3-log2 33 --steps 1 --warmup 0 --no-cpu-baseline)
timeout -k 10 240 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_VALU \
  SQ_WAVE_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d "$OUT/issue" -o run -- "${CMD[@]}" \
  > "$OUT/issue.bench.json" 2> "$OUT/issue.err"
timeout -k 10 240 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_THREAD_CYCLES_VALU \
  SQ_WAVES SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 --output-format csv -d "$OUT/mix" -o run -- "${CMD[@]}" \
  > "$OUT/mix.bench.json" 2> "$OUT/mix.err"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- "${CMD[@]}" \
  > "$OUT/kt.bench.json" 2> "$OUT/kt.err"
timeout -k 10 400 python3 bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err"
echo done
