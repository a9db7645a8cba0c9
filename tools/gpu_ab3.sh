#!/bin/bash
# GPU tests, then an interleaved A/B of checksum-kernel variants on config 3 (10M packets).
#   tools/gpu_ab3.sh <tag> "<ab cases>" [skip-tests]
set -o pipefail
TAG=${1:-ab3}
OUT=gpurun_out
mkdir -p $OUT
if [ -z "$3" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > "$OUT/${TAG}_gpu_tests.log" 2>&1 || { tail -30 "$OUT/${TAG}_gpu_tests.log"; exit 1; }
  tail -2 "$OUT/${TAG}_gpu_tests.log"
fi
AB_CASES=$2 timeout -k 10 400 python -u tools/ab_kernels.py 10000000 ${AB_ROUNDS:-11} 3 > $OUT/${TAG}_ab_cfg3.log 2>&1 || { tail -20 $OUT/${TAG}_ab_cfg3.log; exit 2; }
cat $OUT/${TAG}_ab_cfg3.log
echo "ab3 ok"
