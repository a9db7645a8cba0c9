# round 3: XCD-contiguous tiles (the blocks of one XCD take one contiguous eighth of the tiles) -- A/B on configs 3, 4, 5
set -o pipefail
mkdir -p gpurun_out
AB_CASES=tile/packed,tile/packed-xcd timeout -k 10 400 python -u tools/ab_kernels.py 10000000 21 3 > gpurun_out/r03y_ab_cfg3.log 2>&1 || { tail -20 gpurun_out/r03y_ab_cfg3.log; exit 1; }
grep -E "median|identical" gpurun_out/r03y_ab_cfg3.log
AB_ML=0 AB_CASES=po/c6,po/c6-xcd timeout -k 10 400 python -u tools/ab_kernels.py 12500000 15 4 > gpurun_out/r03y_ab_cfg4.log 2>&1 || { tail -20 gpurun_out/r03y_ab_cfg4.log; exit 2; }
grep -E "median|identical" gpurun_out/r03y_ab_cfg4.log
AB_ML=12 AB_CASES=po/packed,po/packed-xcd timeout -k 10 400 python -u tools/ab_kernels.py 10000000 15 5 > gpurun_out/r03y_ab_cfg5.log 2>&1 || { tail -20 gpurun_out/r03y_ab_cfg5.log; exit 3; }
grep -E "median|identical" gpurun_out/r03y_ab_cfg5.log
