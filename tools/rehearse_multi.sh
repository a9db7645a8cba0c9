#!/bin/bash
# Multi-rank rehearsal of bench.py's N>1 path on a one-GPU box: 2 ranks over gloo sharing the card (shards, the
# timing barrier / MAX, config 4's per-rank flow tables gathered and merged on rank 0). Not a scaling measurement.
#   tools/rehearse_multi.sh <tag>  -> gpurun_out/<tag>_rehearse_cfg*.json
set -o pipefail
TAG=${1:-rh}
mkdir -p gpurun_out
for c in 4 3; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port $((29500 + c)) bench.py --gpus 2 --config $c --packets 2000000 --steps 5 --warmup 2 \
    --dist-backend gloo --no-traffic > gpurun_out/${TAG}_rehearse_cfg$c.json 2> gpurun_out/${TAG}_rehearse_cfg$c.err || exit 1
  tail -1 gpurun_out/${TAG}_rehearse_cfg$c.json | cut -c1-400
done
