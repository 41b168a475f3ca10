# Address-search A/B over both key modes: the address GPU tests on the default library, then the
# addrgen leg (deterministic and random keys, 3 null bytes) alternating the default library and
# variants/<name> on the same box.   usage: tools/addr_ab_modes.sh OUTTAG variant
set -e
OUT=gpurun_out/${1:?tag}
V=${2:?variant}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_addressgen.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_addr.log 2>&1
tail -1 $OUT/pytest_addr.log
for mode in det random; do
  for v in default $V default $V; do
    if [ $v = default ]; then L=pybitmessage_amd/lib/libbmpow_hip.so; else L=variants/$v/libbmpow_hip.so; fi
    BMPOW_LIB=$L timeout -k 10 200 python3 bench.py --config addrgen --addr-mode $mode --null-bytes 3 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/addr_${mode}_$v.json
    python3 -c "import json;d=json.load(open('$OUT/addr_${mode}_$v.json'));print('$mode $v', d['value'], d['kernel']['tries_per_s'])"
  done
done
