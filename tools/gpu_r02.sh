#!/bin/bash
# Round-2 GPU-box check (repo root): GPU tests, then the default bench line and a kernel-trace summary.
#   tools/gpu_r02.sh <tag>   -> gpurun_out/<tag>_*
set -o pipefail
TAG=${1:-r02}
OUT=gpurun_out
ROOT=$(pwd)
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > "$OUT/${TAG}_gpu_tests.log" 2>&1 || { tail -30 "$OUT/${TAG}_gpu_tests.log"; exit 1; }
tail -3 "$OUT/${TAG}_gpu_tests.log"
timeout -k 10 300 python -u bench.py --cpu-seconds 5 > "$OUT/${TAG}_bench.json" 2> "$OUT/${TAG}_bench.err" || exit 2
cat "$OUT/${TAG}_bench.json"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/${TAG}_prof" -o bench --output-format csv -- \
  python3 "$ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-e2e \
  > "$ROOT/$OUT/${TAG}_prof_bench.json" 2> "$ROOT/$OUT/${TAG}_prof.err" || exit 3
echo "gpu r02 ok"
