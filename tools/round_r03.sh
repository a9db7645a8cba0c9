#!/bin/bash
# Round-3 measurement of the current tree on the GPU box (repo root), in two calls:
#   tools/round_r03.sh <tag> tests   -> the whole -m gpu suite, smoke(), PMC traffic per config
#   tools/round_r03.sh <tag> bench   -> every config's bench line (with that traffic) + kernel-trace summaries
set -o pipefail
TAG=${1:-r03}
PART=${2:-tests}
CFGS=${3:-"3 5 4 2"}
OUT=gpurun_out
mkdir -p "$OUT"
if [ "$PART" = tests ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread \
    > "$OUT/${TAG}_gpu_tests.log" 2>&1 || { tail -40 "$OUT/${TAG}_gpu_tests.log"; exit 1; }
  tail -2 "$OUT/${TAG}_gpu_tests.log"
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/${TAG}_smoke.log" 2>&1 || { tail -20 "$OUT/${TAG}_smoke.log"; exit 2; }
  cat "$OUT/${TAG}_smoke.log"
  tools/measure_traffic.sh "$TAG" "$CFGS" > "$OUT/${TAG}_traffic.log" 2>&1 || { tail -20 "$OUT/${TAG}_traffic.log"; exit 3; }
  cat "$OUT"/${TAG}_traffic_cfg*.json | grep -E '"config"|hbm_bytes|write_bytes'
else
  tools/bench_all.sh "$TAG" "$CFGS" > "$OUT/${TAG}_bench_all.log" 2>&1 || { tail -20 "$OUT/${TAG}_bench_all.log"; exit 4; }
  cat "$OUT/${TAG}_bench_all.log"
fi
echo "round r03 $PART ok"
