#!/bin/bash
# PMC passes over the A/B harness (run on the GPU box from the repo root); each --pmc pass is its own run.
# usage: AB_CASES=... tools/pmc.sh <outdir> <packets> <rounds> <config> "<pass1 counters>" "<pass2 counters>" ...
set -o pipefail
OUT=$1; N=$2; R=$3; CFG=$4; shift 4
mkdir -p "$OUT"
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$ROOT" || exit 1
i=0
for pass in "$@"; do
  i=$((i + 1))
  # shellcheck disable=SC2086
  timeout -k 10 300 rocprofv3 --pmc $pass -d "$OUT/p$i" -o "p$i" --output-format csv -- \
    python3 tools/ab_kernels.py "$N" "$R" "$CFG" > "$OUT/p$i.log" 2>&1 || exit $?
done
