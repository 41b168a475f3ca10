# round 3: the interleaved (column) work-item layout + cross-shard bound on the GPU: the -m gpu
# suite, shard latency, and C1 / C3 / C2 bench lines.
set -euo pipefail
OUT=gpurun_out/r03c; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m "gpu and not slow" -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
timeout -k 10 200 python3 tools/shard_latency.py > $OUT/shard_latency.json 2> $OUT/shard_latency.err
timeout -k 10 200 python3 bench.py --config c1 --steps 20 --warmup 2 --no-cpu-baseline > $OUT/c1.json 2> $OUT/c1.err
timeout -k 10 200 python3 bench.py --config c3 --c3-log2 36 --steps 1 --warmup 0 --no-cpu-baseline > $OUT/c3.json 2> $OUT/c3.err
timeout -k 10 300 python3 bench.py --config c2 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/c2.json 2> $OUT/c2.err
