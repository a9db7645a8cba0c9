#!/bin/bash
# Interleaved A/B: parse-only product (tight second round + dword-aligned re-gather of stacks past the window) vs the
# tight round without the re-gather (variant 51) and the skip-generic diagnostic (44), config 5; product vs 51 on
# config 4.   tools/ab_realign.sh <tag> [rounds]
set -o pipefail
TAG=${1:-ra}
R=${2:-9}
mkdir -p gpurun_out
AB_ML=12 AB_CASES=po/product,po/norealign,po/skip-generic timeout -k 10 300 python -u tools/ab_kernels.py 10000000 $R 5 > gpurun_out/${TAG}_cfg5.log 2>&1 || exit 1
AB_ML=0 AB_CASES=po/product,po/norealign timeout -k 10 300 python -u tools/ab_kernels.py 12500000 $R 4 > gpurun_out/${TAG}_cfg4.log 2>&1 || exit 2
for f in gpurun_out/${TAG}_cfg5.log gpurun_out/${TAG}_cfg4.log; do
  echo "== $f"; grep -E "median|identical" "$f"
done
