#!/bin/bash
# PMC HBM traffic of the parse kernel for each bench config (GPU box, repo root): two rocprofv3 --pmc passes
# (FETCH_SIZE, WRITE_SIZE: they do not fit one pass) over bench.py itself, so the numbers belong to exactly the
# launch bench.py times; then gpurun_out/<tag>_traffic_cfg<N>.json, keyed by config / size / records / kernel sha.
#   tools/measure_traffic.sh <tag> "<configs>" [extra bench.py args, e.g. --layout packed]
set -o pipefail
TAG=${1:-tr}
CFGS=${2:-"3"}
shift 2 2>/dev/null
EXTRA="$*"
OUT=gpurun_out
ROOT=$(pwd)
mkdir -p "$OUT"
export TMPDIR=/tmp
cfgargs() {  # "3s512" -> --config 3 --sizes 512
  case "$1" in
    *s*) echo "--config ${1%%s*} --sizes ${1#*s}" ;;
    *) echo "--config $1" ;;
  esac
}
for c in $CFGS; do
  mkdir -p "$OUT/${TAG}_pmc_cfg$c"
  for ctr in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $ctr -d "$ROOT/$OUT/${TAG}_pmc_cfg$c/$ctr" -o p --output-format csv -- \
      python3 "$ROOT/bench.py" $(cfgargs "$c") --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-traffic $EXTRA \
      > "$ROOT/$OUT/${TAG}_pmc_cfg$c/$ctr.json" 2> "$ROOT/$OUT/${TAG}_pmc_cfg$c.$ctr.err") || exit 1
  done
  python3 tools/pmc_traffic.py "$OUT/${TAG}_pmc_cfg$c/FETCH_SIZE" "$OUT/${TAG}_pmc_cfg$c/WRITE_SIZE" \
    "$OUT/${TAG}_pmc_cfg$c/FETCH_SIZE.json" "$OUT/${TAG}_traffic_cfg$c.json" || exit 2
done
echo "traffic ok"
