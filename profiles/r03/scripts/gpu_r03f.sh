# round 3: why a lone C1 object over-hashes on one shard -- column-count sweep (BMPOW_COLUMNS) and the
# single-address atomic rate a block queue would need.
set -euo pipefail
OUT=gpurun_out/r03f; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 120 ./tools/diag/atomic_rate > $OUT/atomic_rate.jsonl 2> $OUT/atomic_rate.err
timeout -k 10 400 python3 tools/diag/c1_columns.py parent 0 1280 1024 768 512 > $OUT/c1_columns.jsonl 2> $OUT/c1_columns.err
timeout -k 10 200 python3 tools/shard_latency.py > $OUT/shard_latency.json 2> $OUT/shard_latency.err
