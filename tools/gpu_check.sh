#!/bin/bash
# GPU-box check after a kernel change: parity tests, then interleaved A/B timing (tools/ab_kernels.py).
#   tools/gpu_check.sh <tag> [ab cases]   -> gpurun_out/<tag>_*
set -o pipefail
TAG=${1:-chk}
CASES=${2:-tile/ml8/csum,tile/gather-first,diag/tile-read}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > "gpurun_out/${TAG}_gpu_tests.log" 2>&1 || exit 1
AB_CASES="$CASES" timeout -k 10 300 python -u tools/ab_kernels.py 10000000 11 > "gpurun_out/${TAG}_ab.log" 2>&1 || exit 2
echo "gpu check ok"
