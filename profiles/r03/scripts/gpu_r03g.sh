# round 3: the per-item block queue (in-order block hand-out) on the GPU -- C1 waste by column count,
# shard latency, C3/C1 bench lines, then the search-path GPU tests.
set -euo pipefail
OUT=gpurun_out/r03g; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python3 tools/diag/c1_columns.py parent 0 1024 512 > $OUT/c1_columns.jsonl 2> $OUT/c1_columns.err
timeout -k 10 200 python3 tools/shard_latency.py > $OUT/shard_latency.json 2> $OUT/shard_latency.err
timeout -k 10 200 python3 bench.py --config c3 --c3-log2 36 --steps 1 --warmup 0 --no-cpu-baseline > $OUT/c3.json 2> $OUT/c3.err
timeout -k 10 200 python3 bench.py --config c1 --steps 20 --warmup 2 --no-cpu-baseline > $OUT/c1.json 2> $OUT/c1.err
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_len.py -m "gpu and not slow" -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
