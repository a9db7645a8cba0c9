#!/bin/bash
# GPU tests, then config 3 / 5 bench lines with the host-to-host legs, then the gather-only A/B.
#   tools/gpu_probe2.sh <tag> "<ab cases>"
set -o pipefail
TAG=${1:-probe}
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$OUT/${TAG}_gpu_tests.log" 2>&1 || { tail -40 "$OUT/${TAG}_gpu_tests.log"; exit 1; }
tail -2 "$OUT/${TAG}_gpu_tests.log"
for c in 3 5; do
  timeout -k 10 300 python -u bench.py --config $c --cpu-seconds 2 > "$OUT/${TAG}_bench_cfg$c.json" 2> "$OUT/${TAG}_bench_cfg$c.err" || exit 2
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'], d['e2e_host_to_host'])" "$OUT/${TAG}_bench_cfg$c.json"
done
tools/ab_parse_only.sh "$TAG" "$2" || exit 3
echo "probe2 ok"
