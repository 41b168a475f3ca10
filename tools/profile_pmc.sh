#!/bin/bash
# PMC passes for bm_search_kernel on the GPU box (one counter group per rocprofv3 run, no
# tracing domains beside --pmc).  Workload: C3 sweep (target 0, fixed initialHash) of
# 2^LOG2 nonces = 2^(LOG2-28) full launches of 2^28 trials each (--step-trials: the PMC method
# stays at 2^28-trial launches whatever the library default).  BMPOW_ONE=0 sends the C3 sweep through
# the engine's bm_search_kernel (the default bench's kernel) rather than run()'s bm_search1_kernel;
# BMPOW_LIB selects a variant build (tools/cmp_variants.sh's variants/<name>).
#   usage: [BMPOW_LIB=variants/x/libbmpow_hip.so] tools/profile_pmc.sh OUTDIR [LOG2]
set -euo pipefail
OUT=${1:?outdir}
LOG2=${2:-33}
mkdir -p "$OUT"
export TMPDIR=/tmp
# PMC_ONE=1: run()'s single-object kernel (bm_search1_kernel) on the same sweep instead
if [ -n "${PMC_ONE:-}" ]; then export BMPOW_ONE=1; else export BMPOW_ONE=0; fi
md5sum "${BMPOW_LIB:-pybitmessage_amd/lib/libbmpow_hip.so}" > "$OUT/lib.md5"
python3 tools/lib_code_md5.py "${BMPOW_LIB:-pybitmessage_amd/lib/libbmpow_hip.so}" > "$OUT/code.md5"
CMD=(python3 bench.py --config c3 --c3-log2 "$LOG2" --steps 1 --warmup 0 --no-cpu-baseline --step-trials 268435456)
if [ -n "${PMC_DEFAULT_BENCH:-}" ]; then CMD=(python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline); fi
pass() {
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- "${CMD[@]}" \
    > "$OUT/$name.bench.json" 2> "$OUT/$name.err"
}
# PASSES: a subset of "instr issue valu fetch write kt" (default: all)
want() { [ -z "${PASSES:-}" ] || [[ " $PASSES " == *" $1 "* ]]; }
if want instr; then pass instr SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM GRBM_GUI_ACTIVE; fi
if want issue; then pass issue SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_BUSY_CU_CYCLES SQ_INSTS_VALU SQ_WAVE_CYCLES \
  SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE; fi
if want valu; then pass valu SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE; fi
if want fetch; then pass fetch FETCH_SIZE; fi
if want write; then pass write WRITE_SIZE; fi
if want kt; then timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- "${CMD[@]}" \
  > "$OUT/kt.bench.json" 2> "$OUT/kt.err"; fi
echo "pmc passes done: $OUT"
