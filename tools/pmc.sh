#!/bin/bash
# PMC passes over the A/B harness (run on the GPU box from the repo root). Each --pmc pass is its own run.
# usage: tools/pmc.sh <outdir> <packets> <rounds> [config]
set -o pipefail
OUT=${1:-gpurun_out/pmc}; N=${2:-2000000}; R=${3:-3}; CFG=${4:-3}
mkdir -p "$OUT"
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$ROOT" || exit 1
run() {  # name, counters...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" -d "$OUT/$name" -o "$name" --output-format csv -- \
    python3 tools/ab_kernels.py "$N" "$R" "$CFG" > "$OUT/$name.log" 2>&1
}
run sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY || exit $?
run sq2 SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH || exit $?
run fetch FETCH_SIZE || exit $?
run write WRITE_SIZE || exit $?
run tcc TCC_HIT_sum TCC_MISS_sum || exit $?
