set -e
mkdir -p gpurun_out/cmp
for v in default v5 i64 default; do
  if [ $v = default ]; then L=pybitmessage_amd/lib/libbmpow_hip.so; else L=build/$v/libbmpow_hip.so; fi
  BMPOW_LIB=$L timeout -k 10 120 python3 bench.py --config c3 --c3-log2 35 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/cmp/c3_$v.json
  python3 -c "import json;d=json.load(open('gpurun_out/cmp/c3_$v.json'));r=d['roofline'];print('$v', r['kernel_ghs'], r['avg_launch_ms'])"
done
BMPOW_LIB=pybitmessage_amd/lib/libbmpow_hip.so timeout -k 10 120 python3 bench.py --config c1 --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/cmp/c1_default.json
python3 -c "import json;d=json.load(open('gpurun_out/cmp/c1_default.json'));print('c1', d['value'], d['ms_per_step'], d['wasted_frac'])"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/cmp/pytest.log 2>&1
tail -2 gpurun_out/cmp/pytest.log
