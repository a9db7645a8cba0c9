#!/bin/bash
# A/B of flow_count_kernel shapes (PCPPX_FLOW_SHAPE, kernels.hip launch_flow_count): for each shape the
# device flow table must equal the host group-by (test_gpu_flow_hash_symmetry_and_flow_table), then
# bench config 4. Writes gpurun_out/fs_<shape>_<grid>.json.
set -o pipefail
mkdir -p gpurun_out
for sg in ${FS_SHAPES:-0:0 1:0 1:256 2:0 3:0 3:256 4:0}; do
  s=${sg%%:*}; g=${sg##*:}
  export PCPPX_FLOW_SHAPE=$s
  if [ "$g" != 0 ]; then export PCPPX_FLOW_GRID=$g; else unset PCPPX_FLOW_GRID; fi
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k flow_table > gpurun_out/fs_${s}_${g}_test.log 2>&1 || exit 1
  timeout -k 10 300 python -u bench.py --config 4 --steps 10 --warmup 3 --no-cpu-baseline --no-e2e \
    > gpurun_out/fs_${s}_${g}.json 2> gpurun_out/fs_${s}_${g}.err || exit 2
  echo "shape $s grid $g: $(python -c "import json;d=json.load(open('gpurun_out/fs_${s}_${g}.json'));print(d['ms_per_step'],d['config'].get('kernel_ms'),d['config'].get('flow_kernel_ms'))")"
done
echo "flow shape ab ok"
