#!/bin/bash
# Search kernel at 5 (in-tree) / 6 / 7 / 8 waves per SIMD: C3 rate (2^35 nonces, twice, same box) and
# the VALU issue counters of each (one rocprofv3 pass per variant).
set -euo pipefail
OUT=gpurun_out/r02_waves; mkdir -p $OUT
export TMPDIR=/tmp
tools/cmp_variants.sh $OUT/ab default variants/var_w6 variants/var_w7 variants/var_w8 > $OUT/ab1.txt 2>&1
tools/cmp_variants.sh $OUT/ab default variants/var_w6 variants/var_w7 variants/var_w8 > $OUT/ab2.txt 2>&1
for v in default var_w6 var_w7 var_w8; do
  if [ $v = default ]; then L=pybitmessage_amd/lib/libbmpow_hip.so; else L=variants/$v/libbmpow_hip.so; fi
  BMPOW_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_BUSY_CU_CYCLES SQ_INSTS_VALU \
    GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc_$v/issue -o run -- \
    python3 bench.py --config c3 --c3-log2 31 --steps 1 --warmup 0 --no-cpu-baseline > $OUT/pmc_$v.json 2> $OUT/pmc_$v.err
done
