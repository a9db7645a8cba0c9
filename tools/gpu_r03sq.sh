# round 3 final source: SQ issue counters of the parse kernel for configs 3, 4, 5 (one PMC pass each)
set -o pipefail
for c in 3 4 5; do tools/sq_counters.sh r03sq $c > /dev/null || exit $c; head -9 gpurun_out/r03sq_sq_cfg$c/summary.txt; done
