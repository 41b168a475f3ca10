# Address-search variant comparison on the GPU box: address tests, then the addrgen bench leg for
# the default library and each variants/<name>/libbmpow_hip.so given as arguments.
set -e
OUT=gpurun_out/${ADDR_OUT:-addr}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_addressgen.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
tail -1 $OUT/pytest.log
for v in default "$@"; do
  if [ $v = default ]; then L=pybitmessage_amd/lib/libbmpow_hip.so; else L=variants/$v/libbmpow_hip.so; fi
  BMPOW_LIB=$L timeout -k 10 200 python3 bench.py --config addrgen --null-bytes 3 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/addr_$v.json
  python3 -c "import json;d=json.load(open('$OUT/addr_$v.json'));print('$v', d['value'], d['kernel'])"
done
