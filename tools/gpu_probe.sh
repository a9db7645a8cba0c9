#!/bin/bash
# Probe run (GPU box, repo root): SQ issue counters of configs 5 and 3, then interleaved A/B of parse-only shapes.
#   tools/gpu_probe.sh <tag> "<ab cases>"
set -o pipefail
TAG=${1:-probe}
tools/sq_counters.sh "$TAG" 5 || exit 1
tools/sq_counters.sh "$TAG" 3 || exit 2
tools/ab_parse_only.sh "$TAG" "$2" || exit 3
echo "probe ok"
