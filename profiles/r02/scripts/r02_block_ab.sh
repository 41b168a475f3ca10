#!/bin/bash
# Search kernel with 128- and 64-lane workgroups (5 and 6 waves per SIMD) against the in-tree 256:
# C3 rate (2^35 nonces, twice, same box) and the co-issue counters of each.
set -euo pipefail
OUT=gpurun_out/r02_block; mkdir -p $OUT
export TMPDIR=/tmp
V="variants/var_b128 variants/var_b64 variants/var_b128w6 variants/var_b64w6"
tools/cmp_variants.sh $OUT/ab default $V > $OUT/ab1.txt 2>&1
tools/cmp_variants.sh $OUT/ab default $V > $OUT/ab2.txt 2>&1
for v in default var_b128 var_b64 var_b128w6 var_b64w6; do
  if [ $v = default ]; then L=pybitmessage_amd/lib/libbmpow_hip.so; else L=variants/$v/libbmpow_hip.so; fi
  BMPOW_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_BUSY_CU_CYCLES SQ_INSTS_VALU \
    GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc_$v/issue -o run -- \
    python3 bench.py --config c3 --c3-log2 31 --steps 1 --warmup 0 --no-cpu-baseline > $OUT/pmc_$v.json 2> $OUT/pmc_$v.err
done
