set -euo pipefail
OUT=gpurun_out/r03b; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 ./tools/ubench_mix > $OUT/ubench_mix.jsonl 2> $OUT/ubench_mix.err
timeout -k 10 200 python3 bench.py --config c3 --c3-log2 36 --steps 1 --warmup 0 --no-cpu-baseline > $OUT/c3.json 2> $OUT/c3.err
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_configs.py -m gpu -x -v --timeout 400 --timeout-method thread -k "c2_full or c4_nonce or c5_default" > $OUT/pytest_configs.log 2>&1
