#!/bin/bash
# Interleaved A/B of parse-only kernel shapes (tools/ab variants) on configs 5, 4 and 3 without checksums.
#   tools/ab_parse_only.sh <tag> [cases]   -> gpurun_out/<tag>_ab_cfg*.log
set -o pipefail
TAG=${1:-ab}
C=${2:-"po/product,po/w7,po/w10,po/w9r6"}
mkdir -p gpurun_out
AB_ML=12 AB_CASES=$C timeout -k 10 300 python -u tools/ab_kernels.py 10000000 7 5 > gpurun_out/${TAG}_ab_cfg5.log 2>&1 || exit 1
AB_ML=0 AB_CASES=$C timeout -k 10 300 python -u tools/ab_kernels.py 12500000 7 4 > gpurun_out/${TAG}_ab_cfg4.log 2>&1 || exit 2
AB_ML=8 AB_CASES=$C timeout -k 10 300 python -u tools/ab_kernels.py 10000000 7 3 > gpurun_out/${TAG}_ab_cfg3po.log 2>&1 || exit 3
for f in gpurun_out/${TAG}_ab_cfg5.log gpurun_out/${TAG}_ab_cfg4.log gpurun_out/${TAG}_ab_cfg3po.log; do
  echo "== $f"; grep median "$f"
done
