# Address-search A/B on one GPU box: the address GPU tests on the default library, then the
# addrgen bench leg alternating the default library and variants/<name> (ABAB, same box).
#   usage: tools/addr_ab.sh OUTTAG variant [variant ...]
set -e
OUT=gpurun_out/${1:?tag}
shift
V="${@:?variant}"
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_addressgen.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_addr.log 2>&1
tail -1 $OUT/pytest_addr.log
for v in default $V default $V; do
  if [ $v = default ]; then L=pybitmessage_amd/lib/libbmpow_hip.so; else L=variants/$v/libbmpow_hip.so; fi
  BMPOW_LIB=$L timeout -k 10 200 python3 bench.py --config addrgen --null-bytes 3 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/addr_$v.json
  python3 -c "import json;d=json.load(open('$OUT/addr_$v.json'));print('$v', d['value'], d['kernel'])"
done
