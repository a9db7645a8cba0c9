#!/bin/bash
# One rocprofv3 --pmc pass per (A/B case, counter set), so every kernel variant gets its own numbers.
# usage (GPU box, repo root): tools/pmc_cases.sh <outdir> <packets> <rounds> "<case1,case2,...>" "<counters1>" ["<counters2>" ...]
set -o pipefail
OUT=$1; N=$2; R=$3; CASES=$4; shift 4
mkdir -p "$OUT"
ROOT=$(pwd)
export TMPDIR=/tmp
cd /tmp || exit 1
IFS=',' read -ra CASE_LIST <<< "$CASES"
for c in "${CASE_LIST[@]}"; do
  tag=$(echo "$c" | tr '/' '_')
  mkdir -p "$ROOT/$OUT/$tag"
  i=0
  for pass in "$@"; do
    i=$((i + 1))
    # shellcheck disable=SC2086
    AB_CASES="$c" timeout -k 10 300 rocprofv3 --pmc $pass -d "$ROOT/$OUT/$tag/p$i" -o "p$i" --output-format csv -- \
      python3 "$ROOT/tools/ab_kernels.py" "$N" "$R" "${CFG:-3}" > "$ROOT/$OUT/$tag/p$i.log" 2>&1 || exit 1
  done
  echo "== case $c"
  python3 "$ROOT/tools/pmc_summary.py" "$ROOT/$OUT/$tag"
done
