# round 3: e2e file rates (r03c) and the early-second-window A/B of the checksum instance (config 3)
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_r03c.sh || exit 1
AB_CASES=tile/packed,tile/packed-earlyB,tile/packed-skipgen timeout -k 10 400 python -u tools/ab_kernels.py 10000000 15 3 > gpurun_out/r03d_ab_earlyB.log 2>&1 || { tail -20 gpurun_out/r03d_ab_earlyB.log; exit 2; }
AB_CASES=tile/ml8/csum,tile/earlyB,tile/earlyB-w4 timeout -k 10 400 python -u tools/ab_kernels.py 10000000 15 3 > gpurun_out/r03d_ab_earlyB_fixed.log 2>&1 || { tail -20 gpurun_out/r03d_ab_earlyB_fixed.log; exit 3; }
grep -E "median|identical" gpurun_out/r03d_ab_earlyB.log gpurun_out/r03d_ab_earlyB_fixed.log
