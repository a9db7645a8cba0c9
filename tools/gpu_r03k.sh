# round 3: flow table with 512 / 1024 partitions and smaller merge blocks (tools/ab pcppx_ab_flow_part shapes 4-7)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/ab_flow_part.py 15 > gpurun_out/r03k_ab_flow.log 2>&1 || { tail -20 gpurun_out/r03k_ab_flow.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r03k_ab_flow.log
