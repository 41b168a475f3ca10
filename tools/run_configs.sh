#!/bin/bash
# Every BASELINE config on one GPU (the box gpurun gives us), one JSON line each, plus a
# rocprofv3 kernel-trace of the default bench and of the verification leg.
#   usage: tools/run_configs.sh OUTDIR TAG
set -euo pipefail
OUT=${1:?outdir}
TAG=${2:?tag}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {
  local name=$1 limit=$2; shift 2
  echo "[$(date +%T)] $name" >&2
  timeout -k 10 "$limit" python3 bench.py "$@" > "$OUT/${TAG}_$name.json" 2> "$OUT/${TAG}_$name.err"
}
run c2 300 --config c2 --steps 3 --warmup 1
run c1 120 --config c1 --steps 20 --warmup 2 --no-cpu-baseline
run c3 200 --config c3 --c3-log2 38 --steps 1 --warmup 0 --no-cpu-baseline
run c4 200 --config c4 --steps 1 --warmup 0 --no-cpu-baseline
run c5 200 --config c5 --objects 4096 --steps 1 --warmup 0 --no-cpu-baseline
run verify 200 --config verify --steps 10 --warmup 2
run addrgen 200 --config addrgen --null-bytes 3 --steps 2 --warmup 1 --cpu-seconds 5
echo "[$(date +%T)] rocprof c2" >&2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_prof_c2" -o run -- \
  python3 bench.py --config c2 --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/${TAG}_prof_c2.json" 2> "$OUT/${TAG}_prof_c2.err"
echo "[$(date +%T)] rocprof verify" >&2
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_prof_verify" -o run -- \
  python3 bench.py --config verify --steps 10 --warmup 1 --no-cpu-baseline > "$OUT/${TAG}_prof_verify.json" 2> "$OUT/${TAG}_prof_verify.err"
echo "[$(date +%T)] rocprof addrgen" >&2
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_prof_addrgen" -o run -- \
  python3 bench.py --config addrgen --null-bytes 3 --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/${TAG}_prof_addrgen.json" 2> "$OUT/${TAG}_prof_addrgen.err"
echo "[$(date +%T)] done" >&2
