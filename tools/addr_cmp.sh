# Address-search variant comparison on the GPU box: for the default library and each
# variants/<name>/libbmpow_hip.so given as arguments -- the address tests, the one-time table build
# (first 1-null-byte search in a fresh process), then the addrgen bench leg.
set -e
OUT=gpurun_out/${ADDR_OUT:-addr}
mkdir -p $OUT
for v in default "$@"; do
  if [ $v = default ]; then L=pybitmessage_amd/lib/libbmpow_hip.so; else L=variants/$v/libbmpow_hip.so; fi
  BMPOW_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_addressgen.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_$v.log 2>&1
  echo "$v $(tail -1 $OUT/pytest_$v.log)"
  BMPOW_LIB=$L timeout -k 10 120 python3 -c "
import time
from pybitmessage_amd import _lib, addressgen
_lib.get()
t = time.perf_counter(); addressgen.search_deterministic(b'table build', 1); t1 = time.perf_counter()
addressgen.search_deterministic(b'table built', 1); t2 = time.perf_counter()
print('$v first 1-byte search %.3f s (table build), second %.4f s' % (t1 - t, t2 - t1))"
  BMPOW_LIB=$L timeout -k 10 200 python3 bench.py --config addrgen --null-bytes 3 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/addr_$v.json
  python3 -c "import json;d=json.load(open('$OUT/addr_$v.json'));print('$v', d['value'], d['kernel'])"
done
