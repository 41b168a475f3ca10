set -e
mkdir -p gpurun_out/r01l
timeout -k 10 300 python -u -m pytest tests/test_addressgen.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r01l/pytest.log 2>&1
tail -1 gpurun_out/r01l/pytest.log
for v in default variants/w8; do
  if [ $v = default ]; then L=pybitmessage_amd/lib/libbmpow_hip.so; else L=$v/libbmpow_hip.so; fi
  BMPOW_LIB=$L timeout -k 10 200 python3 bench.py --config addrgen --null-bytes 3 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r01l/addr_$(basename $v).json
  python3 -c "import json;d=json.load(open('gpurun_out/r01l/addr_$(basename $v).json'));print('$v', d['value'], d['kernel'])"
done
timeout -k 10 120 python3 bench.py --config c1 --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/r01l/c1.json
python3 -c "import json;d=json.load(open('gpurun_out/r01l/c1.json'));print('c1', d['value'], d['ms_per_step'], d['wasted_frac'])"
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()"
