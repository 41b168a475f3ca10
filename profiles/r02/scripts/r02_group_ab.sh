#!/bin/bash
# Search kernel with each round's eight bitop3 issued back to back (BM_GROUP_BITOP3) vs in-tree:
# exact answers on 64 C2 objects first (re-hashed on the host), then C3 rate twice and co-issue counters.
set -euo pipefail
OUT=gpurun_out/r02_group; mkdir -p $OUT
export TMPDIR=/tmp
BMPOW_LIB=variants/var_grp/libbmpow_hip.so timeout -k 10 200 python3 bench.py --objects 64 --steps 1 --warmup 0 \
  --no-cpu-baseline > $OUT/c2_64.json 2> $OUT/c2_64.err
tools/cmp_variants.sh $OUT/ab default variants/var_grp > $OUT/ab1.txt 2>&1
tools/cmp_variants.sh $OUT/ab default variants/var_grp > $OUT/ab2.txt 2>&1
for v in default var_grp; do
  if [ $v = default ]; then L=pybitmessage_amd/lib/libbmpow_hip.so; else L=variants/$v/libbmpow_hip.so; fi
  BMPOW_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_BUSY_CU_CYCLES SQ_INSTS_VALU \
    GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc_$v/issue -o run -- \
    python3 bench.py --config c3 --c3-log2 31 --steps 1 --warmup 0 --no-cpu-baseline > $OUT/pmc_$v.json 2> $OUT/pmc_$v.err
done
