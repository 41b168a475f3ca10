#!/bin/bash
# Kernel rate of alternative builds of libbmpow_hip.so (BMPOW_LIB) on the same box.
#   usage: [CONFIGS="c3 c2 c5"] tools/cmp_variants.sh OUTDIR variant...
#   variant = default | variants/<name>, optionally +VAR=value (an environment setting for that leg,
#   e.g. default+BMPOW_ONE=0: C3 through the engine's bm_search_kernel instead of bm_search1_kernel)
# c3: 2^35 nonces, 2 steps; c2: the default bench, 2 steps; c5: a 4,096-object sample, 1 step;
# c5tm: the 100,000-object flood at test-mode difficulty (many hits per block), 1 step.
set -e
OUT=${1:?outdir}; shift
mkdir -p "$OUT"
CONFIGS=${CONFIGS:-c3}
i=0
for vv in "$@"; do
  v=${vv%%+*}; envs=(); [ "$v" = "$vv" ] || envs=(${vv#*+})
  if [ "$v" = default ]; then L=pybitmessage_amd/lib/libbmpow_hip.so; else L=$v/libbmpow_hip.so; fi
  n=$(basename "$v")$( [ ${#envs[@]} -eq 0 ] || echo "_${envs[*]}" | tr ' =' '__')_$i; i=$((i + 1))
  line="$n"
  for c in $CONFIGS; do
    case $c in
      c3) args=(--config c3 --c3-log2 35 --steps 2 --warmup 1) ;;
      c2) args=(--steps 2 --warmup 1) ;;
      c5) args=(--config c5 --objects 4096 --steps 1 --warmup 0) ;;
      c5tm) args=(--config c5 --test-mode --steps 1 --warmup 1) ;;
    esac
    env BMPOW_LIB=$L "${envs[@]}" timeout -k 10 200 python3 bench.py "${args[@]}" --no-cpu-baseline > "$OUT/${c}_$n.json"
    line="$line $(python3 -c "import json;d=json.load(open('$OUT/${c}_$n.json'));r=d['roofline'];print('$c', d['value'], r['kernel_ghs'])")"
  done
  echo "$line"
done
