#!/bin/bash
# Full validation + measurement of the current build: -m gpu suite, PMC passes (C3), rocprof of the
# exact default bench command, C1.
set -euo pipefail
OUT=${1:?outdir}
mkdir -p "$OUT"
export TMPDIR=/tmp
tools/gpu_tests.sh "$OUT"
tools/profile_pmc.sh "$OUT/pmc" 33
python3 tools/pmc_summary.py "$OUT/pmc" > "$OUT/pmc_summary.json"
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_default" -o run -- \
  python3 bench.py > "$OUT/bench_default_prof.json" 2> "$OUT/bench_default_prof.err"
timeout -k 10 200 python3 bench.py --config c1 --steps 20 --warmup 2 --no-cpu-baseline > "$OUT/c1.json" 2> "$OUT/c1.err"
echo done
