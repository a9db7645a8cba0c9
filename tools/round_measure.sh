#!/bin/bash
# Round-end measurement on the GPU box (repo root): GPU tests, PMC traffic of the default kernel,
# the default bench line (with the traffic just measured), a rocprofv3 kernel-trace summary of it, and
# the extra config bench lines (tools/bench_all.sh).
# usage: tools/round_measure.sh <tag>   -> gpurun_out/<tag>_*
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out
ROOT=$(pwd)
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$OUT/${TAG}_gpu_tests.log" 2>&1 || exit 1
AB_FILTER=tile/ml8/csum
timeout -k 10 600 tools/pmc_cases.sh "$OUT/${TAG}_pmc" 10000000 3 "$AB_FILTER" "FETCH_SIZE" "WRITE_SIZE" \
  > "$OUT/${TAG}_pmc.log" 2>&1 || exit 2
python tools/pmc_traffic.py "$OUT/${TAG}_pmc/tile_ml8_csum/p1" "$OUT/${TAG}_pmc/tile_ml8_csum/p2" 10000000 3 8 \
  "$OUT/${TAG}_traffic.json" > /dev/null || exit 3
timeout -k 10 600 python bench.py --traffic "$OUT/${TAG}_traffic.json" > "$OUT/${TAG}_bench.json" 2> "$OUT/${TAG}_bench.err" || exit 4
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/${TAG}_prof" -o bench --output-format csv -- \
  python3 "$ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --traffic "$ROOT/$OUT/${TAG}_traffic.json" \
  > "$ROOT/$OUT/${TAG}_prof_bench.json" 2> "$ROOT/$OUT/${TAG}_prof.err" || exit 5
cd "$ROOT" || exit 6
tools/bench_all.sh "$TAG" "2 4 5" > "$OUT/${TAG}_bench_all.log" 2>&1 || exit 7
echo "round measure ok"
