# round 3: the relay version of the cross-shard bound -- split-window tests, shard latency, C1.
set -euo pipefail
OUT=gpurun_out/r03d; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 200 python3 tools/shard_latency.py > $OUT/shard_latency.json 2> $OUT/shard_latency.err
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_len.py -m "gpu and not slow" -x -v --timeout 300 --timeout-method thread -k "c1_sweep or shard or c4 or layout or random_lengths or nonce_sharding" > $OUT/pytest_gpu.log 2>&1
timeout -k 10 200 python3 bench.py --config c1 --steps 20 --warmup 2 --no-cpu-baseline > $OUT/c1.json 2> $OUT/c1.err
