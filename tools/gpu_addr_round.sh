set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN_TAG:-r01r}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
tail -1 $O/pytest.log
timeout -k 10 200 python3 bench.py --config addrgen --null-bytes 3 --steps 2 --warmup 1 --cpu-seconds 5 > $O/addrgen.json 2> $O/addrgen.err
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_addrgen -o run -- python3 bench.py --config addrgen --null-bytes 3 --steps 1 --warmup 1 --no-cpu-baseline > $O/prof_addrgen.json 2> $O/prof_addrgen.err
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()"
