#!/bin/bash
# GPU-box check after a kernel change (repo root): the GPU tests, then one bench line per config given.
#   tools/gpu_quick.sh <tag> "<configs>" [pytest args]   -> gpurun_out/<tag>_*
set -o pipefail
TAG=${1:-q}
CFGS=${2:-"3"}
shift 2
OUT=gpurun_out
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread "$@" \
  > "$OUT/${TAG}_gpu_tests.log" 2>&1 || { tail -40 "$OUT/${TAG}_gpu_tests.log"; exit 1; }
tail -2 "$OUT/${TAG}_gpu_tests.log"
for c in $CFGS; do
  timeout -k 10 300 python -u bench.py --config "$c" --no-cpu-baseline --no-e2e > "$OUT/${TAG}_bench_cfg$c.json" \
    2> "$OUT/${TAG}_bench_cfg$c.err" || { tail -5 "$OUT/${TAG}_bench_cfg$c.err"; exit 2; }
  python - "$OUT/${TAG}_bench_cfg$c.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = d["config"]; r = d["roofline"]
print(f"cfg {c['workload'][:40]}: {d['ms_per_step']} ms/step kernel {c['kernel_ms']} ms  frac {r['frac']}  {d['value']} Mpps  flow {c.get('flow_table', {}).get('flow_kernel_ms')}")
PY
done
