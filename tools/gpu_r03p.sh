# round 3: flow table with block-local queue segments (tools/ab pcppx_ab_flow_part shape 8) vs the product (shape 5 = 0)
set -o pipefail
mkdir -p gpurun_out
AB_SHAPES=0,5,8 timeout -k 10 400 python -u tools/ab_flow_part.py 15 > gpurun_out/r03p_ab_flow.log 2>&1 || { tail -20 gpurun_out/r03p_ab_flow.log; exit 5; }
grep -v amdgpu.ids gpurun_out/r03p_ab_flow.log
