# Large-comb width A/B: the default library (24-bit) against variants/w26 (-DAR_WBITS_LARGE=26).
mkdir -p gpurun_out/s4_w26
for v in default w26; do
  if [ $v = default ]; then L=pybitmessage_amd/lib/libbmpow_hip.so; W=24; else L=variants/w26/libbmpow_hip.so; W=26; fi
  BMPOW_LIB=$L timeout -k 10 200 python3 -c "
import time
from pybitmessage_amd import _lib, addressgen
lib = _lib.get()
assert lib.bmpow_addr_set_comb($W) >= 0, lib.bmpow_last_error()
t = time.perf_counter(); addressgen.search_deterministic(b'table build', 1); tb = time.perf_counter() - t
pp = b'bmpow address-search benchmark rank 0'
f = addressgen.search_deterministic(pp, 3)
t = time.perf_counter()
for _ in range(3): f = addressgen.search_deterministic(pp, 3)
el = time.perf_counter() - t
print('$v comb', lib.bmpow_addr_last_comb(), 'build %.3f s' % tb, 'k', f.k, 'tries/s %.1f M' % (3 * (f.k + 1) / el / 1e6))
" || exit 1
done
BMPOW_LIB=variants/w26/libbmpow_hip.so timeout -k 10 300 python -u -m pytest tests/test_addressgen.py -m gpu -x -q -k "large_comb" --timeout 200 > gpurun_out/s4_w26/pytest.log 2>&1; tail -1 gpurun_out/s4_w26/pytest.log
