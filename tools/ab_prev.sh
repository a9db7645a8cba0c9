#!/bin/bash
# Interleaved A/B of today's product kernels against tools/ab/prev (an earlier product tree rebuilt from git):
# parse-only on configs 5 and 4, checksums on config 3.   tools/ab_prev.sh <tag> [rounds]
set -o pipefail
TAG=${1:-prev}
R=${2:-9}
mkdir -p gpurun_out
AB_ML=12 AB_CASES=po/product,po/prev timeout -k 10 300 python -u tools/ab_kernels.py 10000000 $R 5 > gpurun_out/${TAG}_cfg5.log 2>&1 || exit 1
AB_ML=0 AB_CASES=po/product,po/prev timeout -k 10 300 python -u tools/ab_kernels.py 12500000 $R 4 > gpurun_out/${TAG}_cfg4.log 2>&1 || exit 2
AB_CASES=tile/ml8/csum,prev/ml8/csum timeout -k 10 300 python -u tools/ab_kernels.py 10000000 $R 3 > gpurun_out/${TAG}_cfg3.log 2>&1 || exit 3
for f in gpurun_out/${TAG}_cfg5.log gpurun_out/${TAG}_cfg4.log gpurun_out/${TAG}_cfg3.log; do
  echo "== $f"; grep median "$f"
done
