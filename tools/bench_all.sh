#!/bin/bash
# Bench lines for every BASELINE config on one GPU (repo root, GPU box) + kernel-trace summaries.
# Uses gpurun_out/<tag>_traffic_cfg<N>.json (tools/measure_traffic.sh <tag>) when present.
#   tools/bench_all.sh <tag> [configs]   -> gpurun_out/<tag>_bench_cfg<N>.json, <tag>_prof_cfg<N>/
set -o pipefail
TAG=${1:-r01}
CFGS=${2:-"3 2 4 5"}
OUT=gpurun_out
ROOT=$(pwd)
mkdir -p "$OUT"
tr() { [ -f "$ROOT/$OUT/${TAG}_traffic_cfg$1.json" ] && echo "--traffic $ROOT/$OUT/${TAG}_traffic_cfg$1.json"; }
for c in $CFGS; do
  timeout -k 10 400 python -u bench.py --config "$c" $(tr "$c") > "$OUT/${TAG}_bench_cfg$c.json" 2> "$OUT/${TAG}_bench_cfg$c.err" || exit 1
  echo "cfg $c: $(head -c 300 "$OUT/${TAG}_bench_cfg$c.json")"
done
export TMPDIR=/tmp
cd /tmp || exit 2
for c in $CFGS; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/${TAG}_prof_cfg$c" -o bench --output-format csv -- \
    python3 "$ROOT/bench.py" --config "$c" --steps 20 --warmup 5 --no-cpu-baseline --no-e2e $(tr "$c") \
    > "$ROOT/$OUT/${TAG}_prof_bench_cfg$c.json" 2> "$ROOT/$OUT/${TAG}_prof_cfg$c.err" || exit 3
done
echo "bench all ok"
