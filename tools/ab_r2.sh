#!/bin/bash
# Interleaved A/B: the parse-only product (second gather round up to the deep stack's extent) vs the whole-window
# second round (variant 50) and the pre-L7 kernel (tools/ab/prev), configs 5 and 4.   tools/ab_r2.sh <tag> [rounds]
set -o pipefail
TAG=${1:-r2}
R=${2:-9}
mkdir -p gpurun_out
AB_ML=12 AB_CASES=po/product,po/r2full,po/prev timeout -k 10 300 python -u tools/ab_kernels.py 10000000 $R 5 > gpurun_out/${TAG}_cfg5.log 2>&1 || exit 1
AB_ML=0 AB_CASES=po/product,po/r2full,po/prev timeout -k 10 300 python -u tools/ab_kernels.py 12500000 $R 4 > gpurun_out/${TAG}_cfg4.log 2>&1 || exit 2
for f in gpurun_out/${TAG}_cfg5.log gpurun_out/${TAG}_cfg4.log; do
  echo "== $f"; grep -E "median|identical" "$f"
done
