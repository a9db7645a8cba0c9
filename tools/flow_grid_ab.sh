#!/bin/bash
set -o pipefail
for g in 256 512 1024 2048; do
  PCPPX_FLOW_GRID=$g timeout -k 10 300 python -u bench.py --config 4 --steps 10 --warmup 3 --no-cpu-baseline --no-e2e > gpurun_out/s2s_g$g.json 2>/dev/null || exit 1
done
