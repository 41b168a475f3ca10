# round 3: block queue + stage-then-launch steps -- the whole -m gpu suite, shard latency, default bench.
set -euo pipefail
OUT=gpurun_out/r03h; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m "gpu and not slow" -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
timeout -k 10 200 python3 tools/shard_latency.py > $OUT/shard_latency.json 2> $OUT/shard_latency.err
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/c2.json 2> $OUT/c2.err
