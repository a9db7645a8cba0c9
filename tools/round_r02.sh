#!/bin/bash
# Round-2 measurement of the current tree on the GPU box (repo root): GPU tests, PMC traffic per config,
# then every config's bench line (with that traffic) and its kernel-trace summary.
#   tools/round_r02.sh <tag> [configs]   -> gpurun_out/<tag>_*
set -o pipefail
TAG=${1:-r02}
CFGS=${2:-"3 5 4 2"}
OUT=gpurun_out
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$OUT/${TAG}_gpu_tests.log" 2>&1 || { tail -40 "$OUT/${TAG}_gpu_tests.log"; exit 1; }
tail -2 "$OUT/${TAG}_gpu_tests.log"
tools/measure_traffic.sh "$TAG" "$CFGS" > "$OUT/${TAG}_traffic.log" 2>&1 || { tail -20 "$OUT/${TAG}_traffic.log"; exit 2; }
tools/bench_all.sh "$TAG" "$CFGS" > "$OUT/${TAG}_bench_all.log" 2>&1 || { tail -20 "$OUT/${TAG}_bench_all.log"; exit 3; }
cat "$OUT/${TAG}_bench_all.log"
echo "round r02 ok"
