#!/bin/bash
# Search kernel with s_setprio 2 on every 5th / 2nd / 3rd workgroup vs in-tree: C3 rate and co-issue counters.
set -euo pipefail
OUT=gpurun_out/r02_prio; mkdir -p $OUT
export TMPDIR=/tmp
V="variants/var_p5 variants/var_p2 variants/var_p3"
tools/cmp_variants.sh $OUT/ab default $V > $OUT/ab1.txt 2>&1
tools/cmp_variants.sh $OUT/ab default $V > $OUT/ab2.txt 2>&1
for v in default var_p5 var_p2 var_p3; do
  if [ $v = default ]; then L=pybitmessage_amd/lib/libbmpow_hip.so; else L=variants/$v/libbmpow_hip.so; fi
  BMPOW_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_BUSY_CU_CYCLES SQ_INSTS_VALU \
    GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc_$v/issue -o run -- \
    python3 bench.py --config c3 --c3-log2 31 --steps 1 --warmup 0 --no-cpu-baseline > $OUT/pmc_$v.json 2> $OUT/pmc_$v.err
done
