# PMC instruction/busy passes of ar_search_kernel for the default library and variants/<name>.
#   usage: tools/pmc_addr_ab.sh OUTDIR variant
set -euo pipefail
OUT=${1:?outdir}
V=${2:?variant}
export TMPDIR=/tmp
for v in default $V; do
  if [ $v = default ]; then export BMPOW_LIB=pybitmessage_amd/lib/libbmpow_hip.so; else export BMPOW_LIB=variants/$v/libbmpow_hip.so; fi
  bash tools/profile_pmc_addr.sh "$OUT/$v"
done
