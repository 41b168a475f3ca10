#!/bin/bash
# Round-2 measurement pass: PMC (C3) incl. VALU issue counters, rocprof of the exact default bench
# command, C5 batch vs PowService, C1, and the new GPU tests.
set -euo pipefail
OUT=${1:?outdir}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
  -k "mixed_kinds or session_add or powservice" > "$OUT/pytest_new.log" 2>&1
tools/profile_pmc.sh "$OUT/pmc" 33
python3 tools/pmc_summary.py "$OUT/pmc" > "$OUT/pmc_summary.json"
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_default" -o run -- \
  python3 bench.py > "$OUT/bench_default_prof.json" 2> "$OUT/bench_default_prof.err"
timeout -k 10 300 python3 bench.py --config c5 --objects 4096 --steps 1 --warmup 1 --no-cpu-baseline \
  > "$OUT/c5_batch.json" 2> "$OUT/c5_batch.err"
timeout -k 10 300 python3 bench.py --config c5 --objects 4096 --steps 1 --warmup 1 --no-cpu-baseline --service \
  > "$OUT/c5_service.json" 2> "$OUT/c5_service.err"
timeout -k 10 200 python3 bench.py --config c1 --steps 20 --warmup 2 --no-cpu-baseline > "$OUT/c1.json" 2> "$OUT/c1.err"
echo done
