#!/bin/bash
# SQ issue counters of the bench kernels for one bench config (GPU box, repo root): one rocprofv3 --pmc pass (at most
# 8 SQ counters per pass).
#   [SQ_COUNTERS="..."] tools/sq_counters.sh <tag> <config>   -> gpurun_out/<tag>_sq_cfg<N>/ + summary on stdout
set -o pipefail
TAG=$1; C=$2
ROOT=$(pwd)
export TMPDIR=/tmp
CTRS=${SQ_COUNTERS:-"SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD"}
case "$C" in
  *s*) CA="--config ${C%%s*} --sizes ${C#*s}" ;;
  *) CA="--config $C" ;;
esac
mkdir -p "gpurun_out/${TAG}_sq_cfg$C"
(cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $CTRS -d "$ROOT/gpurun_out/${TAG}_sq_cfg$C" -o p --output-format csv -- \
  python3 "$ROOT/bench.py" $CA --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-traffic \
  > "$ROOT/gpurun_out/${TAG}_sq_cfg$C/bench.json" 2> "$ROOT/gpurun_out/${TAG}_sq_cfg$C/err.log") || exit 1
python3 tools/pmc_summary.py "gpurun_out/${TAG}_sq_cfg$C" | tee "gpurun_out/${TAG}_sq_cfg$C/summary.txt"
