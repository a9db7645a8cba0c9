#!/bin/bash
# Flow-table check (GPU box, repo root): flow / filter GPU tests, then config 4's bench line and kernel-trace summary.
#   tools/gpu_flow.sh <tag>
set -o pipefail
TAG=${1:-flow}
OUT=gpurun_out
ROOT=$(pwd)
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "flow or filter" \
  > $OUT/${TAG}_tests.log 2>&1 || { tail -30 $OUT/${TAG}_tests.log; exit 1; }
tail -1 $OUT/${TAG}_tests.log
timeout -k 10 300 python -u bench.py --config 4 --no-cpu-baseline --no-e2e > $OUT/${TAG}_bench_cfg4.json 2> $OUT/${TAG}_bench_cfg4.err || exit 2
python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['ms_per_step'], d['config']['kernel_ms'], d['config']['flow_table'])" $OUT/${TAG}_bench_cfg4.json
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/${TAG}_prof4 -o b --output-format csv -- \
  python3 $ROOT/bench.py --config 4 --steps 20 --warmup 5 --no-cpu-baseline --no-e2e > $ROOT/$OUT/${TAG}_prof4.json 2> $ROOT/$OUT/${TAG}_prof4.err) || exit 3
echo "flow ok"
